// The fused fcnet update of peer mode (ddrl_ppo_update_peer): the row half of this context's
// rank, exchanging its LSB-tagged partial quads with the peer context's launch through shared
// outboxes with system-scope buffer stores and loads (sc0 sc1), as launch_update_ffn_peer
// (ppo_ffn_impl.h, DDRL_FFN_AT = 2).  The norm exchange between the rank's two branches stays
// inside the launch (relaxed system-scope atomics, as the atomic protocol).
#define DDRL_FFN_AT 2
#include "ppo_ffn_impl.h"
