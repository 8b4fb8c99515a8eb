"""GPU idle time between kernels from a rocprofv3 kernel trace (csv):
    python tools/timeline_gaps.py <kernel_trace.csv> [--skip 0.4] [--top 25]
Reports, over the trace after the first `skip` fraction of kernels (warm-up), the busy fraction (union of
kernel intervals), the idle time by gap size, and the largest gaps with the kernels on either side."""
import argparse
import csv
import re


def short(n):
    n = re.sub(r'\(.*', '', n)
    n = re.sub(r'^void ', '', n)
    return n[:60]


ap = argparse.ArgumentParser()
ap.add_argument('csv')
ap.add_argument('--skip', type=float, default=0.4)
ap.add_argument('--top', type=int, default=25)
ap.add_argument('--window', type=int, default=0)
a = ap.parse_args()
rows = list(csv.DictReader(open(a.csv)))
ks = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows)
ks = ks[int(len(ks) * a.skip):]
t0, t1 = ks[0][0], max(k[1] for k in ks)
busy, end, gaps = 0, ks[0][0], []
prev = None
for s, e, n in ks:
    if s > end:
        gaps.append((s - end, prev, n))
    busy += max(0, e - max(s, end))
    end = max(end, e)
    prev = n
span = t1 - t0
print('kernels %d  span %.2f ms  busy %.2f ms (%.1f %%)  idle %.2f ms' % (len(ks), span / 1e6, busy / 1e6,
                                                                       100 * busy / span, (span - busy) / 1e6))
for lo, hi in ((0, 5e3), (5e3, 2e4), (2e4, 1e5), (1e5, 1e12)):
    g = [x[0] for x in gaps if lo <= x[0] < hi]
    print('  gaps %7.0f-%-9.0f ns: %5d, %.2f ms' % (lo, min(hi, 9e9), len(g), sum(g) / 1e6))
agg = {}
for g, p, n in gaps:
    k = (short(p), short(n))
    c = agg.setdefault(k, [0, 0])
    c[0] += 1
    c[1] += g
print('idle by (before -> after), top %d:' % a.top)
for k, (c, g) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
    print('  %8.3f ms %5d x  %s -> %s' % (g / 1e6, c, k[0], k[1]))

# context of the largest gaps
big = sorted([(s - e, i) for i, ((s, e2, n), (_, e, _)) in enumerate(zip(ks[1:], ks[:-1]))], reverse=True)[:2]
for g, i in big:
    print('--- gap %.3f ms after kernel %d' % (g / 1e6, i))
    for j in range(max(0, i - 8), min(len(ks), i + 8)):
        s, e, n = ks[j]
        print('   %12.3f us  dur %9.3f us  %s' % ((s - ks[i][1]) / 1e3, (e - s) / 1e3, short(n)))

# per kernel: launches, mean duration, and the idle gap before it, over the gaps shorter than 100 us (within a step)
per = {}
for j in range(1, len(ks)):
    s, e, n = ks[j]
    g = s - max(k[1] for k in ks[max(0, j - 4):j])
    c = per.setdefault(short(n), [0, 0, 0, 0])
    c[0] += 1
    c[1] += e - s
    if 0 < g < 1e5:
        c[2] += g
        c[3] += 1
print('per kernel: launches, mean duration, total, mean idle gap before it (gaps < 100 us)')
for n, (c, d, g, ng) in sorted(per.items(), key=lambda kv: -kv[1][1])[:a.top]:
    print('  %6d  %9.2f us  %9.3f ms  gap %7.2f us  %s' % (c, d / c / 1e3, d / 1e6, g / max(ng, 1) / 1e3, n))

# one window of consecutive kernels from the middle of the trace (a block's launch sequence)
if a.window:
    m = len(ks) // 2
    print('--- %d kernels from the middle: start relative to the previous end, duration' % a.window)
    for j in range(m, min(len(ks), m + a.window)):
        s, e, n = ks[j]
        print('   gap %9.2f us  dur %8.2f us  %s' % ((s - ks[j - 1][1]) / 1e3, (e - s) / 1e3, short(n)))
