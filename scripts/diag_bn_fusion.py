"""Localise a BN-fusion gradient mismatch: one SGD step of ResNet-50 (batch 4) under
several fusion settings, per-parameter relative difference of the updates against the
unfused graph (worst parameters first)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
import test_bn_fusion_gpu as T  # noqa: E402

VARIANTS = [('base', {'HETU_FUSE_BN_BWD': '0'}),
            ('bwd', {'HETU_FUSE_BN_BWD': '1'}),
            ('bwd_nomask', {'HETU_FUSE_BN_BWD': '1', 'HETU_BN_MASKED_STORE': '0'}),
            ('no_s2', {'HETU_FUSE_BN_BWD': '0', 'HETU_S2_JOIN': '0'}),
            ('bwd_no_s2', {'HETU_FUSE_BN_BWD': '1', 'HETU_S2_JOIN': '0'})]
res = {}
for name, env in VARIANTS:
    for k in ('HETU_BN_MASKED_STORE', 'HETU_S2_JOIN'):
        os.environ.pop(k, None)
    os.environ.update({k: v for k, v in env.items() if k != 'HETU_FUSE_BN_BWD'})
    l, d, nf = T._resnet_step(env['HETU_FUSE_BN_BWD'] == '1', False)
    res[name] = (l, d)
    print(name, 'loss', l, 'fused', nf, flush=True)
l0, d0 = res['base']
for name in res:
    if name == 'base':
        continue
    l, d = res[name]
    num = sum(float((d[k] - d0[k]).norm()) ** 2 for k in d0)
    den = sum(float(d0[k].norm()) ** 2 for k in d0)
    rows = sorted(((float((d[k] - d0[k]).norm() / d0[k].norm().clamp_min(1e-12)), k) for k in d0
                   if float(d0[k].norm()) > 0), reverse=True)
    print('%-12s loss %.6f vs %.6f  total rel %.4f' % (name, l, l0, (num / den) ** 0.5))
    for e, k in rows[:8]:
        print('    %.4f %s' % (e, k))
