// The fused fcnet update's KSP = 1 kernels (one workgroup per branch: the data-parallel gradient
// launches of at most 64 rows, DDRL_UPDATE_SPLIT=1), as launch_update_ffn_k1 (ppo_ffn_impl.h,
// DDRL_FFN_KSP = 1), built with the default scheduling flags; launch_update_ffn forwards them.
#define DDRL_FFN_KSP 1
#include "ppo_ffn_impl.h"
