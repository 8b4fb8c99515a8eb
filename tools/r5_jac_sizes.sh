# fc JAC launch duration against grid size (tools/r5_jac_sizes.py under a kernel trace); summary per grid size
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_jac
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o jac -- python3 $R/tools/r5_jac_sizes.py > $O/run.log 2>&1
cd $R
python3 - <<'EOF'
import csv, glob, collections
f = glob.glob('gpurun_out/r5_jac/tr/**/*kernel_trace.csv', recursive=True)[0]
by = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'fcnet_h3_kernel' in r['Kernel_Name']:
        g = int(r.get('Grid_Size_X', r.get('Grid_Size', 0))) // int(r.get('Workgroup_Size_X', r.get('Workgroup_Size', 1)))
        by[g].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000.0)
out = []
for g in sorted(by):
    v = sorted(by[g])[5:-5] or by[g]
    out.append('workgroups %5d  samples %6d  launches %3d  median %.1f us  min %.1f us' % (g, g * 16, len(by[g]), v[len(v) // 2], min(by[g])))
open('gpurun_out/r5_jac/summary.txt', 'w').write('\n'.join(out) + '\n')
print('\n'.join(out))
EOF
