#!/bin/bash
# r04: phase timeline of the C5 GNN step (diagnostic build), MPNN and GAT1 layers.
set -o pipefail
mkdir -p gpurun_out/gst
DDRL_LIB= timeout -k 10 240 python -u tools/diag_gnn_stamps.py 2048 mpnn > gpurun_out/gst/mpnn.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/diag_gnn_stamps.py 2048 gat1 > gpurun_out/gst/gat1.log 2>&1 || exit 1
