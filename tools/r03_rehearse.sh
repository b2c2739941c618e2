#!/bin/bash
# multi-GPU paths rehearsed on one GPU: 2 ranks (gloo, both on device 0) and one
# process driving 8 shards of configs[3] on device 0
set -o pipefail
TAG=${1:-r03r}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 2 --dist-backend gloo --one-device --steps 10 --warmup 2 --no-cpu-baseline > $O/n2.json 2> $O/n2.err &&
python3 -c "import json; d=json.loads(open('$O/n2.json').read().strip().splitlines()[-1]); print('n2', d['value'], d['n_gpus'], d['parity_vs_reference'], {k: (v.get('value'), v.get('parity_vs_reference')) for k, v in d['methods'].items() if 'cfg3' in k})" &&
timeout -k 10 300 python -u bench.py --multi-context 8 --one-device --steps 10 --warmup 2 --no-cpu-baseline --no-configs > $O/mc8.json 2> $O/mc8.err &&
python3 -c "import json; d=json.loads(open('$O/mc8.json').read().strip().splitlines()[-1]); print('mc8', {k: (v.get('value'), v.get('parity_vs_reference')) for k, v in d['methods'].items() if 'cfg3' in k})"
echo "rc=$?"
