#!/bin/bash
# round-4 call 40: the driver's command on the final tree, repeated -- `python
# bench.py` (defaults) three times and `--warmup 3` twice: headline spread
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04ao}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
for L in d1 d2 d3 w3a w3b; do
  case $L in w3*) A="--warmup 3" ;; *) A="" ;; esac
  timeout -k 10 600 python3 -u bench.py $A > $O/$L.json 2> $O/$L.err || exit 1
  python3 -c "import json; d=json.load(open('$O/$L.json')); print('$L', d['warmup'], d['value'], d['ms_per_step'], d['methods']['ches_batch_resident']['value'], d['methods']['cfg1_pippenger_2^16_batch_c14']['value'], d['valu_roofline']['mad_frac'], d['parity_vs_reference'])"
done
echo "done $(date +%T)"
