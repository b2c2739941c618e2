# G2 2^20 standalone: config_file_n_exp_20 (beta 0) vs _beta (q = 2^20, h = 13), alternating, same box
set -o pipefail
O=gpurun_out/r05g2c; mkdir -p $O
for b in 0 1 0 1 0 1; do
  timeout -k 10 400 python -u bench.py --group 2 --beta $b --no-configs --no-cpu-baseline --no-shards > $O/b.json 2> $O/b.err || exit 1
  echo "## G2 --beta $b" >> $O/ab.txt
  python tools/bench_summary.py $O/b.json 2>&1 | sed -n 1,3p >> $O/ab.txt
done
cat $O/ab.txt
