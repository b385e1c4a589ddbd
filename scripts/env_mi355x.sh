#!/bin/bash
# Site setup for MI355X nodes (reference: scripts/config_crusher.sh / config_summit.sh module
# loads + MPIPreferences).  No MPI is needed: torch.distributed (gloo) is the control plane and
# RCCL over xGMI the data plane.  Source this before building or running.
export ROCM_PATH=${ROCM_PATH:-/opt/rocm}
export PATH=$ROCM_PATH/bin:$PATH
export LD_LIBRARY_PATH=$ROCM_PATH/lib:${LD_LIBRARY_PATH:-}
export HSA_ENABLE_IPC_MODE_LEGACY=0      # dmabuf IPC (RCCL / CUDA-tensor sharing across ranks)
export ARCH=${ARCH:-gfx950}
# one OpenMP thread per rank unless the CPU backend is used on its own
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-1}
# RCCL: keep the defaults (xGMI peer-to-peer); uncomment to debug
# export NCCL_DEBUG=INFO
repo=$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)
export PYTHONPATH=$repo:${PYTHONPATH:-}
