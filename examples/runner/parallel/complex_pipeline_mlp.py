"""Hand-built pipeline (reference examples/runner/parallel/complex_pipeline_mlp.py,
SURVEY §2.3 S9): every rank builds ONLY its own stage, wiring the stages by hand
with ``pipeline_send_op`` / ``pipeline_receive_op`` and differentiating its
stage with ``gradients(..., insert_grad=<received output gradient>)``.

    rank 0      x -> layers -> send(act, 1);   recv(grad, 1) -> backward -> update
    rank 1..N-2 recv(act) -> layers -> send(act);  recv(grad) -> backward -> update,
                send(d act_in) back
    rank N-1    recv(act) -> layers -> loss -> backward -> update, send(d act_in) back

The MLP, weights and batch are the ones of ``mlp_parallel.py``, so the per-step
losses must reproduce ``results/base.npy`` (``validate_results.py``).  Messages
are RCCL send/recv over xGMI on GPUs, gloo on CPU (shapes travel in a header,
reference executor.py:774-833).

    python bin/heturun -w 2 python examples/runner/parallel/complex_pipeline_mlp.py
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', '..', '..'))
sys.path.insert(0, HERE)
import hetu_61a7_amd as ht  # noqa: E402
from mlp_parallel import weights, batch  # noqa: E402


def stage_layers(nl, rank, world):
    return list(range(nl))[rank * nl // world:(rank + 1) * nl // world]


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--batch-size', type=int, default=64)
    p.add_argument('--steps', type=int, default=5)
    p.add_argument('--lr', type=float, default=0.05)
    p.add_argument('--out', default=os.path.join(HERE, 'results'))
    a = p.parse_args(argv)

    comm = ht.wrapped_mpi_nccl_init()
    rank, world = comm.myRank.value, comm.nRanks.value
    ws = weights()
    nl = len(ws)
    assert 2 <= world <= nl, 'one stage per rank, at most %d stages' % nl
    import torch
    ctx = ht.gpu(comm.localRank.value) if torch.cuda.is_available() else ht.cpu(0)
    opt = ht.optim.SGDOptimizer(a.lr)

    def layer(h, i):
        W = ht.Variable(name='w%d' % i, value=ws[i], ctx=ctx)
        if i == 1:
            h = ht.matmul_op(h, W, ctx=ctx)
        else:
            b = ht.Variable(name='b%d' % i, value=np.zeros(ws[i].shape[1], np.float32), ctx=ctx)
            h = ht.linear_op(h, W, b, ctx=ctx)
        return ht.relu_op(h, ctx=ctx) if i < nl - 1 else h

    x = y_ = loss = None
    if rank == 0:
        x = ht.Variable(name='x', trainable=False, ctx=ctx)
        h = x
    else:
        act_in = ht.pipeline_receive_op(rank - 1, comm, ctx=ctx)
        h = act_in
    for i in stage_layers(nl, rank, world):
        h = layer(h, i)
    if rank == world - 1:
        y_ = ht.Variable(name='y_', trainable=False, ctx=ctx)
        loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(h, y_, ctx=ctx), [0], ctx=ctx)
        out, insert = loss, None
    else:
        send_act = ht.pipeline_send_op(h, rank + 1, comm, ctx=ctx)
        out, insert = h, ht.pipeline_receive_op(rank + 1, comm, ctx=ctx)
    params = opt.get_var_list(out)
    opt.params = params
    wrt = params if rank == 0 else [act_in] + params
    grads = ht.gradients(out, wrt, insert_grad=insert)
    train = ht.optim.OptimizerOp(grads if rank == 0 else grads[1:], opt)
    # evaluation order is the schedule (reference order): the forward send must
    # come before anything that waits on the returning gradient
    evals = [loss] if loss is not None else []
    if rank < world - 1:
        evals.append(send_act)
    if rank > 0:
        evals.append(ht.pipeline_send_op(grads[0], rank - 1, comm, ctx=ctx))
    evals.append(train)
    ex = ht.Executor(evals, ctx=ctx)

    X, Y = batch(a.batch_size)
    feed = {}
    if x is not None:
        feed[x] = X
    if y_ is not None:
        feed[y_] = Y
    losses = []
    for _ in range(a.steps):
        res = ex.run(feed_dict=feed, convert_to_numpy_ret_vals=True)
        if loss is not None:
            losses.append(float(np.mean(res[0])))
    if losses:
        os.makedirs(a.out, exist_ok=True)
        path = os.path.join(a.out, 'manual_pp_rank%d.npy' % rank)
        np.save(path, np.asarray(losses, np.float64))
        print('rank %d manual pipeline losses %s -> %s' % (rank, ' '.join('%.5f' % v for v in losses), path),
              flush=True)
    from hetu_61a7_amd.parallel import comm as C
    C.destroy()
    return losses


if __name__ == '__main__':
    main()
