#!/bin/bash
# Does the rayon shape's speed depend on the NUMA node of the host memory?
# tools/rayon_probe.py with the process pinned to each node's CPUs in turn.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python tools/numa_info.py > gpurun_out/numa_info.json; cat gpurun_out/numa_info.json
python -c "import torch; p=torch.cuda.get_device_properties(0); print('gpu pci', getattr(p,'pci_bus_id',None), getattr(p,'pci_device_id',None), getattr(p,'pci_domain_id',None))"
nodes=$(ls -d /sys/devices/system/node/node[0-9]* | sed 's/.*node//' | tr '\n' ' ')
for i in 1 2; do
  for n in $nodes any; do
    if [ $n = any ]; then e="X=1"; else e="PROBE_NODE=$n"; fi
    env $e PROBE_MODES=pinned PROBE_REPS=3 timeout -k 10 200 python -u tools/rayon_probe.py \
        > gpurun_out/numa_${n}_$i.json 2> gpurun_out/numa_${n}_$i.err
    rc=$?; echo "node $n run $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python -c "import json; d=json.load(open('gpurun_out/numa_${n}_$i.json')); print(d['link_floor_ms'], d['seen_pinned'], d['fresh_pinned'])"
  done
done
