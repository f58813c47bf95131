#!/bin/bash
# Build a tuning variant of libfsm.so with extra -D flags (run here, not on the GPU box):
#   tools/build_variant.sh NAME -DFSM_TSR_EPT=4 ...   ->  spark-fsm_amd/build/var/NAME/libfsm.so
# Load it with FSM_LIB_PATH=spark-fsm_amd/build/var/NAME/libfsm.so for A/B runs.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
out=$R/spark-fsm_amd/build/var/$name
make -s -C "$R/spark-fsm_amd" HOSTDBG="$*" OUT="$out/libfsm.so" OBJDIR="$out/obj"
echo "$out/libfsm.so"
