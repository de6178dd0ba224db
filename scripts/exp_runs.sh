set -e
mkdir -p gpurun_out/exp
for e in ${EXPS:-2 3 4}; do
  FSG_LIB=$PWD/fluvio_amd/_lib/libfsg_exp$e.so timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/exp/exp$e.log 2>&1 || true
done
