/* ABI layout probe (tests/test_binding.py): sizeof / offsetof of every field
 * of the C-ABI structures, as the C compiler lays them out, one line each:
 * "<struct> <field> <offset> <size>" and "<struct> SIZEOF <size> <size>". */
#include <stddef.h>
#include <stdio.h>

#include "ikgrasp.h"

#define F(S, f) printf("%s %s %zu %zu\n", #S, #f, offsetof(S, f), sizeof(((S*)0)->f))
#define Z(S) printf("%s SIZEOF %zu %zu\n", #S, sizeof(S), sizeof(S))

int main(void) {
  F(ikg_model_desc, nq); F(ikg_model_desc, parent); F(ikg_model_desc, axis); F(ikg_model_desc, placement);
  F(ikg_model_desc, lower); F(ikg_model_desc, upper); F(ikg_model_desc, root_q); F(ikg_model_desc, arm_q);
  F(ikg_model_desc, hand); F(ikg_model_desc, hook); Z(ikg_model_desc);
  F(ikg_params, eps); F(ikg_params, dt); F(ikg_params, max_iters); F(ikg_params, variant);
  F(ikg_params, lambda); F(ikg_params, problems_per_wave); F(ikg_params, check_collision); Z(ikg_params);
  F(ikg_collision_desc, n_geoms); F(ikg_collision_desc, kind); F(ikg_collision_desc, joint);
  F(ikg_collision_desc, placement); F(ikg_collision_desc, dims); F(ikg_collision_desc, target_geom);
  F(ikg_collision_desc, n_pairs); F(ikg_collision_desc, pairs); Z(ikg_collision_desc);
  F(ikg_frame_kin_out, placement); F(ikg_frame_kin_out, velocity); F(ikg_frame_kin_out, J);
  F(ikg_frame_kin_out, dJ); F(ikg_frame_kin_out, dJv); F(ikg_frame_kin_out, err); F(ikg_frame_kin_out, derr);
  Z(ikg_frame_kin_out);
  return 0;
}
