#!/bin/bash
# build_variant.sh NAME "EXTRA FLAGS" -- an in-tree build of libmofhip with
# extra compile definitions, as mofhip/libmofhip_NAME.so (A/B measurements
# on one box: MOFHIP_LIB=<that path> python bench.py ...)
set -e
name=$1; extra=$2
cd "$(dirname "$0")/../manifold-based-optical-flow-method_amd/csrc"
make -j8 BUILD=build_$name OUT=../mofhip/libmofhip_$name.so \
    CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 $extra" >/dev/null
echo "built mofhip/libmofhip_$name.so ($extra)"
