"""MoE model family (reference examples/moe/test_moe_top.py:17-36, test_moe_hash.py,
test_moe_ktop1.py, test_moe_sam.py, test_moe_base.py).

``moe_top`` is the reference's top-k benchmark network: one MoE layer (TopK gate,
``num_local_experts`` two-layer ReLU experts per GPU, expert-parallel over all
ranks with RCCL all-to-all) followed by reduce-sum over the model dim, softmax
over tokens and an NLL loss, plus the balance loss.
"""
from __future__ import annotations

import numpy as np

from .. import ops as ht
from ..layers.moe import (TopKGate, KTop1Gate, HashGate, SAMGate, DenseToSparseGate, BalanceAssignmentGate,
                          Expert, MoELayer, KTop1Layer, HashLayer, SAMLayer)


def moe_experts(model_dim, hidden_size, num_local_experts, rank=0, dropout_rate=0.1):
    return [Expert(embed_dim=model_dim, ffn_dim=hidden_size, dropout_rate=dropout_rate, activation='relu',
                   name='expert_%d' % (rank * num_local_experts + i)) for i in range(num_local_experts)]


def moe_top(x, y_, batch_size, num_tokens, model_dim, hidden_size, num_local_experts, world=1, rank=0,
            top=2, gate='topk', dropout_rate=0.1, hash_ids=None, temperature=None):
    """Returns (loss, y).  ``x`` [B, T, d]; ``y_`` the NLL targets [B]."""
    E = num_local_experts * world
    ntok = batch_size * num_tokens
    experts = moe_experts(model_dim, hidden_size, num_local_experts, rank, dropout_rate)
    extra = []
    if gate == 'topk':
        out = MoELayer(TopKGate(model_dim, ntok, E, k=top), experts, num_tokens, model_dim, world, top=top)(x)
    elif gate == 'dts':
        out = MoELayer(DenseToSparseGate(model_dim, ntok, E, k=top, temperature=temperature), experts, num_tokens,
                       model_dim, world)(x)
    elif gate == 'ktop1':
        out = KTop1Layer(KTop1Gate(model_dim, ntok, E, k=top), experts, num_tokens, model_dim, world, k=top)(x)
    elif gate == 'sam':
        out = SAMLayer(SAMGate(model_dim, ntok, E, k=top, num_local_gpus=max(world, 1)), experts, num_tokens,
                       model_dim, world, k=top, num_local_gpus=max(world, 1))(x)
    elif gate == 'hash':
        out = (HashLayer(HashGate(model_dim, ntok, E), experts, num_tokens, model_dim, world)(x, hash_ids),)
    elif gate == 'base':
        out = (MoELayer(BalanceAssignmentGate(model_dim, ntok, E, device_id=rank), experts, num_tokens, model_dim,
                        world, name='BalanceAssignmentLayer')(x),)
    else:
        raise ValueError(gate)
    y, extra = out[0], list(out[1:])
    y = ht.array_reshape_op(y, [-1, num_tokens, model_dim])
    y = ht.reduce_sum_op(y, axes=2)
    y = ht.softmax_op(y)
    loss = ht.nll_loss_op(y, y_, num_tokens)
    for e in extra:
        loss = loss + e
    return loss, y


def moe_top_bench(args, world, rank, local):
    """Benchmark step for BASELINE config 5: the reference's top-2 script
    (examples/moe/scripts/run_top2.sh:1 -- test_moe_top.py --top=2 --num_local_experts=2
    --batch_size=64; 1024 tokens per sequence, d_model = d_ffn = 2048, expert dropout
    0.1, SGD lr 0.125), bf16 compute.  Gate: top-k (default) or the dense-to-sparse gate
    (``--moe-gate dts``: its temperature anneals once per step and the JSON reports the
    budget / active experts per token of the last step read).
    Returns (step_fn, samples_per_step, config, metric, finish_fn); a "sample"
    is one token."""
    import torch
    import hetu_61a7_amd as H
    B, T, d, ffn = args.batch or 64, 1024, 2048, 2048
    nle = int(getattr(args, 'moe_local_experts', 2) or 2)
    gate = getattr(args, 'moe_gate', 'topk')
    sched = getattr(args, 'dts_schedule', None)
    temp = None
    if gate == 'dts' and sched:
        from ..layers.moe import DTSTemperature
        tau0, decay, tau_min = (float(v) for v in sched.split(','))
        temp = DTSTemperature(tau0=tau0, tau_min=tau_min, decay=decay)
    x, y_ = H.Variable(name='x', trainable=False), H.Variable(name='y_', trainable=False)
    loss, y = moe_top(x, y_, B, T, d, ffn, nle, world, rank, top=2, gate=gate, temperature=temp)
    train = H.optim.SGDOptimizer(learning_rate=0.125).minimize(loss)
    kw = dict(mixed_precision=args.dtype, seed=1234)
    if world > 1:
        ex = H.Executor({'train': [loss, train]}, ctx=H.gpu(local), comm_mode='AllReduce', **kw)
    else:
        ex = H.Executor({'train': [loss, train]}, ctx=H.gpu(local), **kw)
    dev = torch.device('cuda', local)
    g = torch.Generator(device=dev)
    g.manual_seed(2000 + rank)
    dt = torch.bfloat16 if args.dtype == 'bf16' else torch.float32
    X = torch.randn((B, T, d), generator=g, device=dev).to(dt)
    Y = torch.zeros((B,), dtype=torch.float32, device=dev)
    feed = {x: X, y_: Y}

    def step():
        ex.run('train', feed_dict=feed)

    if gate == 'dts':
        from ..ops.moe_dts import DTSGatingOp
        g = [n for n in ex.subexecutor['train'].topo_order if isinstance(n, DTSGatingOp)][0]

        timeline = []      # (step, budget, ms): per-step timing of the schedule run

        def step():
            import time
            if sched:
                torch.cuda.synchronize()
                t0, b0 = time.perf_counter(), g.budget
            if g.calls == 0 and g.budget > g.k_min:
                # The budget only shrinks (dense to sparse), and each budget has its own expert
                # capacity, i.e. its own GEMM shapes.  Run one (untimed, first warmup) step at
                # every smaller budget first so that a budget change inside the timed window
                # does not autotune the new shapes there; the histograms of these forced calls
                # are dropped -- they must not steer the real budget.
                keep = g.budget
                for b in range(g.k_min, keep):
                    g.budget = b
                    ex.run('train', feed_dict=feed)
                g.budget = keep
                g._pending, g._tau_at, g.history = [], {}, []
                g.pretuned_budgets = list(range(g.k_min, keep))
                if sched:
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()       # the pretuning steps are not the schedule's
            ex.run('train', feed_dict=feed)
            if sched:
                torch.cuda.synchronize()
                timeline.append((g.calls, b0, (time.perf_counter() - t0) * 1e3))

        def extra():
            h = g.history[-1] if g.history else None
            out = {'steps': g.calls, 'pretuned_budgets': getattr(g, 'pretuned_budgets', []),
                   'tau': round(g.temperature.value, 4), 'budget_k': g.budget,
                   'active_experts_per_token_last': round(h[3], 3) if h else None,
                   'active_experts_first_to_last': [round(x[3], 3) for x in g.history[::max(1, len(g.history) // 8)]]}
            if sched:
                per, changes, prev = {}, [], None
                for call, b, ms in timeline[1:]:          # step 1 carries the pretuning
                    per.setdefault(b, []).append(ms)
                for call, b, ms in timeline:
                    if prev is not None and b != prev:
                        changes.append({'step': call, 'from': prev, 'to': b})
                    prev = b
                out['schedule'] = sched
                out['budget_changes'] = changes
                out['ms_per_step_by_budget'] = {str(b): round(sum(v) / len(v), 3) for b, v in sorted(per.items())}
                out['steps_by_budget'] = {str(b): len(v) for b, v in sorted(per.items())}
                out['tokens_per_s_by_budget'] = {str(b): round(B * T * world * 1e3 / (sum(v) / len(v)), 1)
                                                 for b, v in sorted(per.items())}
            return {'dts': out}
        step.extra = extra

    cfg = {'model': 'MoE %s (examples/moe/test_moe_top.py: d=2048, ffn=2048, %d experts/GPU)'
                    % ('top-2' if gate == 'topk' else gate, nle),
           'global_batch': B * world, 'seq_len': T, 'parallelism': 'ep%d (all-to-all) + dp%d gate' % (world, world),
           'gate': gate, 'experts': nle * world, 'optimizer': 'sgd', 'per_gpu_batch': B}
    return step, B * T * world, cfg, 'tokens/sec (whole node) MoE %s gate, expert all-to-all' % gate, None


def moe_random_batch(batch_size, num_tokens, model_dim, seed=0):
    rng = np.random.RandomState(seed)
    return (rng.normal(size=(batch_size, num_tokens, model_dim)).astype(np.float32),
            np.zeros((batch_size,), np.float32))
