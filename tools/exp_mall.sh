# per-image paired-series time vs batch (memory-side cache residency of d1/d2) + phase stamps, then the k128 parity tests
cd $GRAFT_REPO_ROOT
for B in 8 16 32 64 128; do timeout -k 5 90 python3 tools/series_only.py --scale 0 --batch $B --mfma 2 --reps 5 2>&1 | grep -a "us/term" || exit 1; done
for B in 64 128 256; do timeout -k 5 90 python3 tools/series_only.py --scale 1 --batch $B --mfma 2 --reps 5 2>&1 | grep -a "us/term" || exit 1; done
for S in 0 1; do INFLOW_LIB=gpurun_alt/lib_stamps.so timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 2 --reps 1 2>&1 | grep -a "var3 mode2" | cut -c1-200 || exit 1; done
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "k128 or headline or golden" 2>&1 | tail -3
