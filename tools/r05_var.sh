# tile: sort before the row gather, uploads on a second stream; ring slot size A/B; ABI tests
set -o pipefail
O=gpurun_out/r05gb; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_blst_ches_abi.py tests/test_gpu_pointer_gather.py tests/test_gpu_dropin.py tests/test_gpu_tile_grid.py tests/test_gpu_driver.py -x -q --timeout 300 --timeout-method thread > $O/abi.txt 2>&1 || { tail -30 $O/abi.txt; exit 1; }
tail -1 $O/abi.txt
for env in "MSM_RING_SLOT_MIB=8" "MSM_RING_SLOT_MIB=32" "MSM_RING_SLOT_MIB=4" "MSM_RING_SLOT_MIB=8"; do
  echo "## $env" >> $O/ga.txt
  env $env timeout -k 10 300 python -u tools/tile_timing.py > $O/t.json 2> $O/t.err || exit 1
  grep "\[tile\]" $O/t.err | awk 'NR==3 || NR==4 || NR==11 || NR==12' >> $O/ga.txt
  python -c "import json; d=json.load(open('$O/t.json')); print({k: (v['ms_per_step'], v['ratio_vs_ctx_sync'], v['parity_vs_reference']) for k, v in d.items()})" >> $O/ga.txt
done
cat $O/ga.txt
