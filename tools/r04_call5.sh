#!/bin/bash
# round-4 call 5: 5 front sets / 4 reducer sets in the lane schedule; then the
# lean-doubling study build (tools/ablib/libmsm_lean.so) against the table-row test
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04e}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_pippenger_batch.py tests/test_gpu_ches.py tests/test_gpu_multi.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
echo "pytest rc=$? $(date +%T) $(tail -1 $O/pytest.txt)"; grep -E "FAILED|Error" $O/pytest.txt | head -20
timeout -k 10 300 python3 -u tools/r04_small_trace.py pb16 c17 c18 c19 > $O/small.txt 2>&1 &&
grep -v amdgpu $O/small.txt | cut -c1-200 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof17 -o run -- python3 $R/tools/r04_small_trace.py c17 > $O/prof17.txt 2>&1 && cd $R &&
cp tools/ablib/libmsm_lean.so msm_blst_amd/libmsm_mi355x.so &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_table_rows.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_lean_rows.txt 2>&1
echo "lean rows rc=$?"; grep -E "PASSED|FAILED|rows differ" $O/pytest_lean_rows.txt | head -20
echo "done $(date +%T)"
