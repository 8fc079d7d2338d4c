#!/bin/bash
# Build a variant of libccg.so with extra -D flags into tools/variants/ (tools/timing only).
# usage: tools/build_variant.sh NAME "-DFOO=1 -DBAR=2"
set -e
ROOT=$(cd $(dirname $0)/.. && pwd)
mkdir -p $ROOT/tools/variants
make -s -j8 -C $ROOT/consensusclustr_amd/csrc OUT=$ROOT/tools/variants/libccg_$1.so BUILD=$ROOT/build/var_$1 VARIANT_DEFS="$2"
