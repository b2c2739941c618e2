#!/bin/bash
# round-4 call 31: front priority greatest vs normal through bench.py
# (--warmup 3 / 5, three runs each), small MSMs and G2
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04af}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
for i in 1 2 3; do
  for P in 1 0; do
    for W in 3 5; do
      L=p${P}_w${W}_$i
      MSM_FRONT_PRIO=$P timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline --warmup $W > $O/$L.json 2> $O/$L.err || exit 1
      python3 -c "import json; d=json.load(open('$O/$L.json')); print('$L', d['value'], d['methods']['ches_batch_resident']['value'], d['roofline']['kernel_ms'], d['parity_vs_reference'])"
    done
  done
done
for P in 1 0; do
  MSM_FRONT_PRIO=$P timeout -k 10 300 python3 -u tools/r04_small_trace.py c17 c18 c19 > $O/small_p$P.txt 2>&1 || exit 1
  grep -v amdgpu $O/small_p$P.txt | sed "s/^/p$P /" | cut -c1-120
  MSM_FRONT_PRIO=$P timeout -k 10 400 python3 -u bench.py --group 2 --no-configs --no-cpu-baseline --no-compare > $O/g2_p$P.json 2> $O/g2_p$P.err || exit 1
  python3 -c "import json; d=json.load(open('$O/g2_p$P.json')); print('G2 p$P', d['value'], d['ms_per_step'])"
done
echo "done $(date +%T)"
