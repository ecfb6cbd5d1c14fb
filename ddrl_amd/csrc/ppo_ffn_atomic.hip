// The fused fcnet update with the formally defined exchange protocol: every granule access a
// relaxed system-scope 64-bit atomic (ppo_ffn_impl.h, DDRL_XCHG_IS_ATOMIC), valid for any
// placement of a policy's workgroups.  The context switches to it (launch_update_ffn_atomic)
// when the default protocol's placement assumption fails (capi.cpp: check_placement) or when
// DDRL_XCHG=atomic is set.
#define DDRL_FFN_AT 1
#include "ppo_ffn_impl.h"
