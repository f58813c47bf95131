#!/bin/bash
# Build libfsm.so of an earlier git revision for A/B runs (run here, not on the GPU box):
#   tools/build_rev.sh REV NAME  ->  spark-fsm_amd/build/var/NAME/libfsm.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
rev=$1; name=$2
out=$R/spark-fsm_amd/build/var/$name
mkdir -p "$out"
rm -rf /tmp/rev_$name
git -C "$R" worktree add -f /tmp/rev_$name "$rev" -q
make -s -C /tmp/rev_$name/spark-fsm_amd OUT="$out/libfsm.so" OBJDIR="/tmp/rev_$name/obj" -j8
git -C "$R" worktree remove --force /tmp/rev_$name
echo "$out/libfsm.so"
