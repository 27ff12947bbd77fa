set -e
for i in 1 2; do
for p in 0 -1; do
timeout -k 10 200 python3 bench.py --pitch $p --cpu-baseline off --pcie off --steps 100 > gpurun_out/ab_$p_$i.log 2>&1
python3 -c "import json;d=json.loads(open('gpurun_out/ab_$p_$i.log').read().strip().splitlines()[-1]);print($p, d['value'], d['roofline']['launch_ms'], d['roofline']['launch_ms_by_direction'])"
done; done
