// Every compiled instance of ppo_rc_kernel<KT, KW, KB, S0T, NLT, ACTT, HWT, CWT, DT, NW>
// (ppo_rc_kernel.h), grouped by the translation unit that compiles it (ppo_rc_inst_<g>.hip:
// the groups build in parallel). ppo_rc.hip declares them all extern and picks one per plan.
// Scratch budget of every instance: profiles/r4_kernel_resources.md (all 0).
#pragma once

#define IA_RC_EXTERN(...) extern template __global__ void ppo_rc_kernel<__VA_ARGS__>(PPOArgs, PPORcGeo);
#define IA_RC_INSTANTIATE(...) template __global__ void ppo_rc_kernel<__VA_ARGS__>(PPOArgs, PPORcGeo);

#define IA_RC_GROUP_A(X) \
  X(2,3,1,5,3,2,32,64,0,4) \
  X(2,2,1,1,3,2,32,64,1,4) \
  X(2,5,2,0,0,-1,0,64,-1,4) \
  X(2,5,2,0,0,-1,0,0,-1,4)

#define IA_RC_GROUP_B(X) \
  X(4,6,1,3,3,1,64,64,0,4) \
  X(4,7,1,5,3,1,64,64,0,4) \
  X(2,3,1,5,3,2,32,64,0,8) \
  X(2,3,1,5,3,2,32,32,0,8) \
  X(2,2,1,1,3,2,32,64,1,8)

#define IA_RC_GROUP_C(X) \
  X(4,6,1,-4,3,1,64,64,0,4) \
  X(4,6,1,-4,3,1,64,64,1,4) \
  X(4,6,1,-4,3,2,64,64,0,4) \
  X(4,6,1,-4,3,2,64,64,1,4)

#define IA_RC_GROUP_D(X) \
  X(4,7,1,-8,3,1,64,64,0,4) \
  X(4,7,1,-8,3,1,64,64,1,4) \
  X(4,7,1,-8,3,2,64,64,0,4) \
  X(4,7,1,-8,3,2,64,64,1,4)

#define IA_RC_GROUP_E(X) \
  X(4,12,2,3,3,1,64,32,0,4) \
  X(4,12,2,-4,3,1,64,32,0,4) \
  X(4,12,2,-4,3,1,64,32,1,4) \
  X(4,12,2,-4,3,2,64,32,0,4) \
  X(4,12,2,-4,3,2,64,32,1,4)

#define IA_RC_GROUP_F(X) \
  X(4,14,2,5,3,1,64,32,0,4) \
  X(4,14,2,-8,3,1,64,32,0,4)

#define IA_RC_INSTANCES(X) IA_RC_GROUP_A(X) IA_RC_GROUP_B(X) IA_RC_GROUP_C(X) IA_RC_GROUP_D(X) IA_RC_GROUP_E(X) IA_RC_GROUP_F(X)
