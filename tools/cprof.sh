#!/bin/bash
# Build the phase-timing diagnostic library (gitignored, travels with gpurun).
set -e
cd "$(dirname "$0")/../motion-planning-and-control-for-dual-manipulator-robot_amd/csrc"
mkdir -p ../ikgrasp/_native/abl
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-slp-vectorize -Xarch_device -ffinite-math-only -Xarch_device -fno-signed-zeros -Xarch_device -Wno-nan-infinity-disabled -DIKG_CPROF -I../../include -I. \
  -shared -o ../ikgrasp/_native/abl/libikgrasp_cprof.so ikg_kernels.hip ikg_packed.hip ikg_quad.hip ikg_collision.hip ikg_control.hip ikg_jit.hip ikg_capi.hip -ldl
