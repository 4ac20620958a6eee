"""Drop-in ``utils`` package (see compute_optical_flow.py).

The package path is extended with every other ``utils`` directory on
sys.path (pkgutil.extend_path), so the reference's own modules that are not
replaced here (draw_optical_flow_field, ...) still import when the
reference checkout is on sys.path behind this directory."""
from pkgutil import extend_path

__path__ = extend_path(__path__, __name__)
