"""Diagnostic variants of the 128-pixel VJP kernel (fused313k.hip) for time attribution -- WRONG RESULTS, never
shipped: the product source stays untouched; a patched copy is compiled into gpurun_alt/lib_<name>.so.

    python tools/build_alt_k128.py <name> <variant>[,<variant>...]
      d2l2   d2 read from image 0 / tile 0 for every tile (L2-resident: the HBM burst removed, the loads kept)
      d1l2   the same for d1
      nod2   no d2 loads at all (multiplier 1)
      nod1   no d1 loads at all (multiplier 1)
      dsyncN first-round workgroups of every other CU group start N k-cycles late (desynchronised bursts)
      DNAME=V  #define NAME V ahead of the source (the product's compile-time switches)
      sub    INFLOW_K128_SUBSTAMPS: stamps inside chunk 1 and phase C (results unchanged; sched_barrier fences)
      stamps no patch (the phase stamps only)
Every alternative library is built with INFLOW_PHASE_STAMPS=1 (fused313.hip / fused313k.hip s_memtime stamps at
the phase boundaries, printed per kernel at exit); `python tools/build_alt_k128.py stamps stamps` gives the product
kernels with stamps.  Run with INFLOW_LIB=gpurun_alt/lib_<name>.so (tools/series_only.py).
"""
import os
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C = os.path.join(R, 'implicit-normalizing-flows_amd', 'csrc')
O = os.path.join(R, 'implicit-normalizing-flows_amd', 'lib', '_hip', 'obj')


def patch(src, variants):
    rep = []
    if 'd2l2' in variants:
        rep.append(('const f32x4* q = dptr(a.d2, 8 * c + wid, b);',
                    'const f32x4* q = reinterpret_cast<const f32x4*>(a.d2 + (((0 + (b >> 1)) * 16 + 8 * c + wid) * 2 + (b & 1)) * 1024 + lane * 16);'))
    if 'd1l2' in variants:
        rep.append(('const f32x4* q = dptr(a.d1, 2 * wid + m, b);',
                    'const f32x4* q = reinterpret_cast<const f32x4*>(a.d1 + (((0 + (b >> 1)) * 16 + 2 * wid + m) * 2 + (b & 1)) * 1024 + lane * 16);'))
    if 'nod2' in variants:
        rep.append(('for (int j = 0; j < 4; ++j) d2v[b][j] = q[j];',
                    'for (int j = 0; j < 4; ++j) d2v[b][j] = f32x4{1.f, 1.f, 1.f, 1.f}; (void)q;'))
    if 'nod1' in variants:
        rep.append(('for (int j = 0; j < 4; ++j) d1v[b][j] = q[j];',
                    'for (int j = 0; j < 4; ++j) d1v[b][j] = f32x4{1.f, 1.f, 1.f, 1.f}; (void)q;'))
    for v in variants:
        if v.startswith('dsync'):      # first-round workgroups on half the CUs start D k-cycles late (results unchanged)
            d = int(v[5:]) * 1000
            rep.append(('  KSTAMP(0);\n',
                        '  if (blockIdx.x < 256 && ((blockIdx.x >> 3) & 1)) {\n'
                        '    const unsigned long long t0_ = __builtin_amdgcn_s_memtime();\n'
                        '    while (__builtin_amdgcn_s_memtime() - t0_ < %dull) __builtin_amdgcn_s_sleep(64);\n'
                        '  }\n  KSTAMP(0);\n' % d))
    for v in variants:
        if v.startswith('D') and '=' in v:  # compile-time switch of the product source, e.g. DK128_EARLY_W3=0
            src = '#define %s %s\n' % tuple(v[1:].split('=')) + src
    if 'sub' in variants:
        src = '#define INFLOW_K128_SUBSTAMPS 1\n' + src
    for old, new in rep:
        assert src.count(old) == 1, old
        src = src.replace(old, new)
    return src


def main():
    name, variants = sys.argv[1], sys.argv[2].split(',')
    src = patch(open(os.path.join(C, 'fused313k.hip')).read(), variants)
    tmp = os.path.join(C, '_alt_%s.hip' % name)
    with open(tmp, 'w') as f:
        f.write(src)
    os.makedirs(os.path.join(R, 'gpurun_alt'), exist_ok=True)
    obj = '/tmp/alt_%s.o' % name
    obj2 = '/tmp/alt_%s_fused313.o' % name
    flags = ['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-ffp-contract=fast',
             '-DINFLOW_PHASE_STAMPS=1', '-c']
    try:
        subprocess.run(flags + ['-o', obj, tmp], check=True)
    finally:
        os.remove(tmp)
    subprocess.run(flags + ['-o', obj2, os.path.join(C, 'fused313.hip')], check=True)
    objs = [obj2] + [os.path.join(O, f) for f in sorted(os.listdir(O))
                     if f.endswith('.o') and f not in ('fused313k.o', 'fused313.o')]
    out = os.path.join(R, 'gpurun_alt', 'lib_%s.so' % name)
    subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-shared', '-fPIC', '-o', out, obj] + objs, check=True)
    print('built', out)


if __name__ == '__main__':
    main()
