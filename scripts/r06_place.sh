#!/bin/bash
# Round 6: does a layout's HBM placement mode follow its allocation order in
# the process?  (Round 2 saw "the first three of eight allocations slow".)
# v76 encode over ten layouts allocated in order, in two fresh processes, then
# in a process that first allocates and keeps a 48 GiB pad.  Diagnostic only:
# the bench keeps allocating once.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06place
mkdir -p $O
ST=12288,16384,20480,28672,36864,45056,53248,61440,69632,77824
for run in a b; do
  timeout -k 10 300 python3 tools/kbench.py --variants 76 --stagger $ST --rounds 2 --iters 10 \
      > $O/order_$run.json 2> $O/order_$run.err || { tail $O/order_$run.err; exit 1; }
  echo "run $run done"
done
timeout -k 10 300 python3 tools/kbench.py --variants 76 --stagger $ST --rounds 2 --iters 10 --pad-gib 48 \
    > $O/order_pad48.json 2> $O/order_pad48.err || { tail $O/order_pad48.err; exit 1; }
echo "pad done"
