#!/bin/bash
# Timing-only ablation builds of the kernel library (tools/ablate.py).
set -e
cd "$(dirname "$0")/../motion-planning-and-control-for-dual-manipulator-robot_amd/csrc"
for v in 0 2 4 6; do
  mkdir -p build_abl$v
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-slp-vectorize -DIKG_ABL=$v -I../../include -I. \
    -shared -o ../ikgrasp/_native/abl/libikgrasp_abl$v.so ikg_kernels.hip ikg_packed.hip ikg_capi.hip 2>/dev/null || \
    { mkdir -p ../ikgrasp/_native/abl && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-slp-vectorize -DIKG_ABL=$v -I../../include -I. -shared -o ../ikgrasp/_native/abl/libikgrasp_abl$v.so ikg_kernels.hip ikg_packed.hip ikg_capi.hip; }
  rmdir build_abl$v
done
ls -la ../ikgrasp/_native/abl
