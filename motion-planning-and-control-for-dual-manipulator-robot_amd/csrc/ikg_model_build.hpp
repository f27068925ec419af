// Host-side construction of the kernel model tables from ikg_model_desc
// (shared by the C-ABI and the host emulator).
#pragma once

#include <cstring>

#include "ikg_device.hpp"
#include "ikgrasp.h"

namespace ikg {

inline bool is_identity(const double* R) {
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      if (R[3 * r + c] != (r == c ? 1.0 : 0.0)) return false;
  return true;
}

template <typename T>
inline void build_kmodel(const ikg_model_desc& d, KModel<T>& k) {
  std::memset(&k, 0, sizeof(k));
  const int r = d.root_q;
  for (int i = 0; i < 9; ++i) k.root_R[i] = (T)d.placement[r][i];
  for (int i = 0; i < 3; ++i) k.root_t[i] = (T)d.placement[r][9 + i];
  k.root_lo = (T)d.lower[r];
  k.root_hi = (T)d.upper[r];
  k.root_q = r;
  k.root_axis = d.axis[r];
  k.rot_mask = 0;
  for (int a = 0; a < 2; ++a)
    for (int j = 0; j < IKG_ARM_DOF; ++j) {
      const int q = d.arm_q[a][j];
      for (int i = 0; i < 9; ++i) k.arm_R[a][j][i] = (T)d.placement[q][i];
      for (int i = 0; i < 3; ++i) k.arm_t[a][j][i] = (T)d.placement[q][9 + i];
      k.arm_lo[a][j] = (T)d.lower[q];
      k.arm_hi[a][j] = (T)d.upper[q];
      k.arm_q[a][j] = q;
      k.arm_axis[j] = d.axis[q];
      if (!is_identity(d.placement[q])) k.rot_mask |= 1 << j;
    }
  for (int a = 0; a < 2; ++a) {
    for (int i = 0; i < 9; ++i) k.hand_R[a][i] = (T)d.hand[a][i];
    for (int i = 0; i < 3; ++i) k.hand_t[a][i] = (T)d.hand[a][9 + i];
    for (int i = 0; i < 9; ++i) k.hook_R[a][i] = (T)d.hook[a][i];
    for (int i = 0; i < 3; ++i) k.hook_t[a][i] = (T)d.hook[a][9 + i];
  }
  for (int q = 0; q < d.nq; ++q) {
    k.lo[q] = (T)d.lower[q];
    k.hi[q] = (T)d.upper[q];
  }
  k.nq = d.nq;
  bool used[IKG_MAX_NQ] = {};
  used[r] = true;
  for (int a = 0; a < 2; ++a)
    for (int j = 0; j < IKG_ARM_DOF; ++j) used[d.arm_q[a][j]] = true;
  k.n_passive = 0;
  for (int q = 0; q < d.nq; ++q)
    if (!used[q]) k.passive_q[k.n_passive++] = q;
}


}  // namespace ikg
