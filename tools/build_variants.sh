#!/bin/bash
# Timing-only variant builds of the kernel library (tools/ablate.py times them
# interleaved in one process), built by the Makefile with the shipped per-file
# flags (the packed kernel's max-ILP scheduler) plus the variant's flags, into
# ikgrasp/_native/var/lib_<name>.so.
# usage: tools/build_variants.sh name "extra flags" [name "flags"]...
set -e
cd "$(dirname "$0")/../motion-planning-and-control-for-dual-manipulator-robot_amd/csrc"
mkdir -p ../ikgrasp/_native/var
rm -f ../ikgrasp/_native/var/*.so
make -s build/ikg_jit_src.inc
while [ $# -gt 0 ]; do
  name=$1; flags=$2; shift 2
  make -s -j8 BUILD=build_var_$name EXTRA="$flags" OUT=../ikgrasp/_native/var/lib_$name.so ../ikgrasp/_native/var/lib_$name.so &
done
wait
rm -rf build_var_*
ls ../ikgrasp/_native/var
