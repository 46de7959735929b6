#!/bin/bash
# A/B build of librq: redqueen_amd/librq_NAME.so with extra compiler flags, reusing the
# main build's objects for every source not named (they must not depend on the flags).
# usage: scripts/dev/variant.sh NAME "EXTRA FLAGS" src1.hip [src2 ...]
# Load it with RQ_SO_PATH=$PWD/redqueen_amd/librq_NAME.so (A/B only).
set -euo pipefail
cd "$(dirname "$0")/../../redqueen_amd/csrc"
NAME=$1; EXTRA=$2; shift 2
mkdir -p "build_$NAME"
cp -p build/*.o "build_$NAME/"
for f in "$@"; do rm -f "build_$NAME/$f.o"; done
make -s -j8 BUILD="build_$NAME" OUT="../librq_$NAME.so" EXTRA="$EXTRA"
