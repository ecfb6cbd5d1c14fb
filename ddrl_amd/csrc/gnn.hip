// GraphNet / MPNN ("gnn") kernels -- placeholder launchers until the GNN path lands.
#include "common.h"
#include "kernels.h"

void launch_act_gnn(hipStream_t, const RouteArgs&, const ActArgs&) {}
void launch_update_gnn(hipStream_t, const UpdateArgs*, const UpdateHyper&, int, float, int) {}
void launch_forward_gnn(hipStream_t, const ForwardArgs&) {}
