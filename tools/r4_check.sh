# Parity subset (128-pixel kernels, headline golden, fc nets), then the POWER and CIFAR benches; results under
# gpurun_out/$1 (default r4).
set -e
OUT=gpurun_out/${1:-r4}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "k128 or headline or power or toy or fc" > $OUT/tests.log 2>&1 || { tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 200 python bench.py --config power --steps 5 --warmup 2 > $OUT/bench_power.json 2>/dev/null
timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 20 --warmup 3 > $OUT/bench.json 2>/dev/null
for f in bench_power bench; do
  python - $OUT/$f.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['achieved'], d['roofline']['frac'],
      d['path']['kernel_busy_frac'])
PY
done
