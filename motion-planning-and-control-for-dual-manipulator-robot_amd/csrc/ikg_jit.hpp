// Model-specialised pair kernels compiled at run time with hipRTC (ikg_jit.hip).
//
// The prebuilt library carries one kernel per compile-time specialisation
// (ikg_model_build.hpp choose_spec): a model outside the Nextage pattern reads
// its joint axes, placement rotations and offsets from the model tables at run
// time.  ikg_model_specialize compiles the same pair-layout loop
// (ikg_solve.hpp pair_batch_body) against a compile-time constant copy of one
// model's tables, so every axis, identity placement, zero offset and limit
// folds into the instruction stream.
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "ikg_device.hpp"

namespace ikg {

// One device's loaded module.  `pair_med` exists only for frame-1 models (the
// medium-range trig series of per-problem seeds); the launcher falls back to
// `pair` when it is null, as the prebuilt launcher does.
struct JitKernels {
  hipModule_t module = nullptr;
  hipFunction_t pair = nullptr;
  hipFunction_t pair_med = nullptr;
  hipFunction_t damped = nullptr;
};

// Source of the specialised kernels for one model / dtype.
template <typename T>
std::string jit_source(const KModel<T>& k);

// hipRTC compile for gfx950.  Returns an empty string on success (code filled)
// or the error with the compiler log.
std::string jit_compile(const std::string& src, std::vector<char>& code);

// Load a code object on the current device.
hipError_t jit_load(const std::vector<char>& code, JitKernels& out);
void jit_unload(JitKernels& k);

}  // namespace ikg
