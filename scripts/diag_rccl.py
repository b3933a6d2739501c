"""Step-by-step one-rank run of the in-house RCCL communicator's primitives with a
stack dump if a step stalls (faulthandler), to locate a hang."""
import faulthandler
import os
import socket
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
faulthandler.dump_traceback_later(60, exit=True)
s = socket.socket()
s.bind(('127.0.0.1', 0))
port = s.getsockname()[1]
s.close()
os.environ.update(RANK='0', WORLD_SIZE='1', LOCAL_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                  HETU_USE_CONFIG='0')
import torch  # noqa: E402


def step(name):
    print('%.2f %s' % (time.time() % 1000, name), flush=True)


step('import comm')
from hetu_61a7_amd.parallel import comm as C  # noqa: E402
step('init_process_group')
w = C.init_process_group(use_gpu=True)
step('backend %s' % w.backend)
t = torch.randn(1 << 20, device='cuda')
step('all_reduce sum')
w.all_reduce(t, 'sum')
torch.cuda.synchronize()
step('all_reduce mean')
w.all_reduce(t, 'mean')
torch.cuda.synchronize()
step('async')
w.all_reduce(t, 'sum', async_op=True).wait()
torch.cuda.synchronize()
step('bf16')
u = torch.randn(1000003, device='cuda')
w.all_reduce_bf16(u, async_op=True).wait()
torch.cuda.synchronize()
step('reduce_scatter')
out = torch.empty(4096, device='cuda')
w.reduce_scatter(out, t[:4096])
torch.cuda.synchronize()
step('all_gather')
ag = torch.empty(4096, device='cuda')
w.all_gather(ag, t[:4096])
torch.cuda.synchronize()
step('broadcast')
b = t[:777].clone()
w.broadcast(b, 0)
torch.cuda.synchronize()
step('all_to_all')
a2a = torch.empty(8192, device='cuda')
w.all_to_all(a2a, t[:8192])
torch.cuda.synchronize()
step('batch_p2p')
dst = torch.empty(513, device='cuda')
for x in w.batch_p2p([('send', t[:513].contiguous(), 0), ('recv', dst, 0)]):
    x.wait()
torch.cuda.synchronize()
step('health %s' % w.health())
step('barrier')
w.barrier()
step('destroy')
C.destroy()
step('done')
