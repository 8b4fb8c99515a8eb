"""Mean SQ counters per dispatch of the VJP kernels in rocprofv3 --pmc CSVs (tools/r5_pmc_sq_k.sh), with the derived
fractions: MFMA-busy share of the SIMD cycles, wait / active shares of the wave cycles, mean waves per SIMD.
    python tools/sq_summary.py gpurun_out/r5_sq_k3_s0 [kernel-name substring, e.g. fcblock_kernel]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else None
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        if (pat in k) if pat else ('net313k_kernel<2' in k or 'net313p_kernel' in k):
            agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k, c in agg.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    print(k[:60], {n: round(v) for n, v in sorted(m.items())})
    gui = m.get('GRBM_GUI_ACTIVE')
    if gui:
        per_xcd = gui / 8          # GRBM_GUI_ACTIVE summed over the 8 XCDs
        simd = 256 * 4 * per_xcd
        if 'SQ_VALU_MFMA_BUSY_CYCLES' in m:
            print('  MFMA busy / SIMD-cycles: %.3f' % (m['SQ_VALU_MFMA_BUSY_CYCLES'] / simd))
    if 'SQ_WAVE_CYCLES' in m:
        wc = m['SQ_WAVE_CYCLES']
        print('  wait_inst %.3f  wait_any %.3f  active_inst %.3f (of wave cycles)' % (
            m.get('SQ_WAIT_INST_ANY', 0) / wc, m.get('SQ_WAIT_ANY', 0) / wc, m.get('SQ_ACTIVE_INST_ANY', 0) / wc))
    if 'SQ_LEVEL_WAVES' in m and 'SQ_BUSY_CYCLES' in m:
        print('  level_waves / busy cycles: %.2f' % (m['SQ_LEVEL_WAVES'] / m['SQ_BUSY_CYCLES']))
