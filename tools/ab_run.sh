mkdir -p gpurun_out/ab
for i in 1 2; do
  timeout -k 10 200 python -u tools/exp_batch.py 20 3 > gpurun_out/ab/cur$i.txt 2>&1 || exit 1
  MSM_LIB=$PWD/tools/ablib/libmsm_prev.so timeout -k 10 200 python -u tools/exp_batch.py 20 3 > gpurun_out/ab/prev$i.txt 2>&1 || exit 1
done
echo done
