#!/bin/bash
# round-4 call 35: the host stager's short first piece (2 MiB) vs none
# (MSM_STAGE_FIRST_MB=0) on the drop-in at 2^20 / 2^16, twice each, after the
# drop-in / pool / gather tests
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04aj}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_engine_cache.py tests/test_gpu_pointer_gather.py tests/test_gpu_tile_grid.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc $(date +%T) $(tail -1 $O/pytest.txt)"; grep -E "FAILED|^E " $O/pytest.txt | head -20
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
  for F in 2 0; do
    MSM_STAGE_FIRST_MB=$F timeout -k 10 300 python3 -u tools/dropin_timing.py 20 > $O/d20_f${F}_$i.json 2> $O/d20_f${F}_$i.err || exit 1
    echo "first=$F 2^20 $(cat $O/d20_f${F}_$i.json | cut -c1-120)"
  done
done
echo "done $(date +%T)"
