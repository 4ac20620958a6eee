"""The library's environment switches (csrc/mof_knobs.h): read in one place,
at most eight, each documented in INTEGRATION.md §5; the checkpoint key
keeps exactly the V-changing ones (mofhip/solve.py)."""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "manifold-based-optical-flow-method_amd", "csrc")


def _knob_names():
    src = open(os.path.join(CSRC, "mof_knobs.cpp")).read()
    table = src[src.index("kNames"):src.index("};", src.index("kNames"))]
    return re.findall(r'"(MOF_[A-Z0-9_]+)"', table)


def test_getenv_only_in_the_knob_reader():
    hits = {}
    for name in sorted(os.listdir(CSRC)):
        if name.endswith((".cpp", ".hip", ".h")):
            n = open(os.path.join(CSRC, name)).read().count("getenv")
            if n:
                hits[name] = n
    assert hits == {"mof_knobs.cpp": 1}, hits


def test_knobs_documented_and_few():
    names = _knob_names()
    assert 0 < len(names) <= 8, names
    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    sec = doc[doc.index("## 5. Runtime switches"):]
    for n in names:
        assert "`%s`" % n in sec, n


def test_checkpoint_key_neutral_switches():
    import sys
    sys.path.insert(0, os.path.join(REPO, "manifold-based-optical-flow-method_amd"))
    from mofhip.solve import _KEY_NEUTRAL
    names = set(_knob_names())
    changes_v = {"MOF_SYM_READS", "MOF_AMG_SMOOTH", "MOF_AMG_OMEGA", "MOF_AMG_BSW"}
    assert changes_v <= names
    assert not (changes_v & _KEY_NEUTRAL)
    assert names - changes_v <= _KEY_NEUTRAL
