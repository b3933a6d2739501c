"""Per-op-type time of the Wide&Deep PS step (host 'cpu' timer = issue/host time)."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
from bench import start_ps_server  # noqa: E402

os.environ.setdefault('MASTER_PORT', '29631')
server = start_ps_server(1, 0)
import torch  # noqa: E402
import hetu_61a7_amd as ht  # noqa: E402
from hetu_61a7_amd.models.ctr import wdl_criteo, synthetic_criteo  # noqa: E402

rows = int(os.environ.get('ROWS', '33762577'))
kind = sys.argv[1] if len(sys.argv) > 1 else 'cpu'
xd, xs, y_ = ht.Variable(name='dense_input'), ht.Variable(name='sparse_input'), ht.Variable(name='y_')
loss, y, _, train = wdl_criteo(xd, xs, y_, feature_dimension=rows, embedding_size=128, learning_rate=0.01)
ex = ht.Executor({'train': [loss, train]}, ctx=ht.gpu(0), comm_mode='Hybrid', cstable_policy='LFUOpt',
                 cache_bound=3, bsp=-1, mixed_precision='bf16', seed=1234, timing=kind)
B, nb = 128, 64
dense, sparse, labels = synthetic_criteo(B * nb, rows, seed=100)
D = torch.from_numpy(dense).cuda()
L = torch.from_numpy(labels).cuda()
S = torch.from_numpy(sparse)
for i in range(40):
    sl = slice((i % nb) * B, (i % nb + 1) * B)
    ex.run('train', feed_dict={xd: D[sl], xs: S[sl], y_: L[sl]})
torch.cuda.synchronize()
ex.clearTimer('train')
t0 = time.perf_counter()
for i in range(40):
    sl = slice((i % nb) * B, (i % nb + 1) * B)
    ex.run('train', feed_dict={xd: D[sl], xs: S[sl], y_: L[sl]})
torch.cuda.synchronize()
print('ms/step (timed run)', (time.perf_counter() - t0) * 1e3 / 40)
t = ex.logOut(log_level='type', name='train')
tot = sum(t.values())
for k, v in sorted(t.items(), key=lambda kv: -kv[1])[:30]:
    print('%-45s %8.3f ms/step' % (k, v))
print('sum %.3f' % tot)
from hetu_61a7_amd.ps import worker  # noqa: E402
ex.config.ps_comm.BarrierWorker()
worker.worker_finish()
server.wait(timeout=60)
