#!/bin/bash
# Compile the REFERENCE rabit (read-only tree at $REF, default /root/reference) out of tree into
# build/ref with a minimal dmlc shim, for head-to-head runs of its own speed_test against ours
# (tools/refbuild/compare_speed.py).  Nothing from the reference is copied into this repository;
# the objects land in build/ref (git-ignored).  Prebuilt binaries shipped inside the reference are
# never used: everything is compiled here from its sources.
set -eu
cd "$(dirname "$0")/../.."
REF=${REF:-/root/reference}
OUT=build/ref
mkdir -p "$OUT/shimsub"
SHIM=$PWD/tools/refbuild
# thread_local.h includes "../include/dmlc/base.h": resolve it from an -I directory one level down
ln -sfn "$SHIM/include" "$OUT/include"
FLAGS="-O3 -std=c++11 -fPIC -pthread -I$REF/include -I$SHIM/include -I$OUT/shimsub -w"
CXX=${CXX:-g++}
for f in allreduce_base allreduce_robust engine engine_mock; do
  [ "$OUT/$f.o" -nt "$REF/src/$f.cc" ] || $CXX $FLAGS -c "$REF/src/$f.cc" -o "$OUT/$f.o"
done
$CXX $FLAGS "$REF/test/speed_test.cc" "$OUT/allreduce_base.o" "$OUT/allreduce_robust.o" \
  "$OUT/engine.o" -o "$OUT/speed_test"
$CXX $FLAGS "$REF/test/speed_test.cc" "$OUT/allreduce_base.o" "$OUT/allreduce_robust.o" \
  "$OUT/engine_mock.o" -o "$OUT/speed_test_mock"
echo "built $OUT/speed_test"
