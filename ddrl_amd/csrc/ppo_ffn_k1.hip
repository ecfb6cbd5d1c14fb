// The fcnet update kernels other than the fused row split, as launch_update_ffn_k1
// (ppo_ffn_impl.h, DDRL_FFN_KSP = 1): KSP = 1 (one workgroup per branch: data-parallel gradient
// launches of at most 64 rows, DDRL_UPDATE_SPLIT=1) and the gradient-export launches of the
// data-parallel loop, built with the default scheduling flags; launch_update_ffn forwards them.
#define DDRL_FFN_KSP 1
#include "ppo_ffn_impl.h"
