"""Model-parallel lowering of ``ht.dispatch`` annotations (the pass the
reference's Dispatch op anticipates but never implements: SURVEY §0.2, §2.3
S10; API of ``gpu_ops/Dispatch.py:34-48`` and the test matrix of
``examples/runner/parallel/test_mlp_mp.py``).

Semantics (SPMD, one process per GPU, the whole job is one model-parallel
group of P ranks): every node outside a tuple context is *replicated* on all
ranks; inside a tuple context, ``dispatch(node, parts)`` declares how a value
is partitioned.  For ``C = matmul(dispatch(A, (pm, pk)), dispatch(B, (pk, pn)))``
the P = pm*pk*pn ranks form a (m, k, n) mesh; rank (im, ik, in) computes
``A[im, ik] @ B[ik, in]``, which is partial over the k axis.

The pass rewrites the forward graph BEFORE autodiff, inserting four collective
ops whose gradients are each other's conjugates, so backward comes out of the
ordinary ``gradients()``:

  MPSlice    replicated -> shard (local slice)      grad: MPGather
  MPGather   shard -> replicated (all-gather)       grad: MPSlice
  MPCopy     identity (operand replicated over an   grad: all-reduce over that axis
             axis it is consumed under)
  MPReduce   partial -> replicated (all-reduce)     grad: identity

(the last two are the "f"/"g" conjugate pair of tensor-parallel layers).  Every
collective runs over an RCCL sub-communicator of the ranks that differ only in
the named mesh axes; all sub-groups are created collectively on every rank.
Supported inside a region: matmul (2-D, all split combinations), unary
elementwise ops, binary elementwise ops between equally-split operands and
bias broadcast.  Region exits gather the value back to a replicated tensor.
"""
from __future__ import annotations

import itertools
from typing import Dict, Optional, Tuple

import torch

from ..ops.node import Op
from ..context import DeviceGroup, dist_env

AXES = ('m', 'k', 'n')


class Mesh(object):
    def __init__(self, sizes: Dict[str, int]):
        self.sizes = {a: int(sizes.get(a, 1)) for a in AXES}
        self.P = self.sizes['m'] * self.sizes['k'] * self.sizes['n']

    def coord(self, rank):
        s = self.sizes
        im, rest = divmod(rank, s['k'] * s['n'])
        ik, inn = divmod(rest, s['n'])
        return {'m': im, 'k': ik, 'n': inn}

    def rank_of(self, c):
        s = self.sizes
        return (c['m'] * s['k'] + c['k']) * s['n'] + c['n']

    def group(self, rank, axes):
        """Ranks sharing rank's coordinates on every axis not in ``axes``."""
        c = self.coord(rank)
        out = []
        for vals in itertools.product(*[range(self.sizes[a]) if a in axes else [c[a]] for a in AXES]):
            out.append(self.rank_of(dict(zip(AXES, vals))))
        return tuple(sorted(out))

    def key(self):
        return tuple(self.sizes[a] for a in AXES)


_COMMS = {}
PENDING_MESHES = []


def _comm(ranks):
    if len(ranks) <= 1:
        return None
    return _COMMS.get(tuple(ranks))


def create_groups(meshes, world):
    """Collective: create every sub-communicator any rank may use, same order
    on all ranks (torch.distributed.new_group is collective over the world)."""
    from . import comm as C
    if world <= 1:
        return
    want = []
    for mesh in meshes:
        for axes in [a for r in range(1, 4) for a in itertools.combinations(AXES, r)]:
            for rank in range(world):
                g = mesh.group(rank, axes)
                if len(g) > 1 and g not in want:
                    want.append(g)
    for g in sorted(want):
        if g not in _COMMS:
            _COMMS[g] = C.new_group_comm(list(g))


def _rank():
    return dist_env()[0]


# ---- collective ops ------------------------------------------------------------------------
class MPSliceOp(Op):
    """Replicated -> this rank's shard. dims: {tensor_dim: mesh_axis}."""

    def __init__(self, node, mesh, dims, ctx=None):
        super().__init__(MPSliceOp, [node], ctx)
        self.mesh, self.dims = mesh, dict(dims)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        c = self.mesh.coord(_rank())
        for d, ax in self.dims.items():
            n = self.mesh.sizes[ax]
            size = x.shape[d] // n
            x = x.narrow(d, c[ax] * size, size)
        return x.contiguous()

    def gradient(self, output_grad):
        return [MPGatherOp(output_grad, self.mesh, self.dims, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        s = list(input_shapes[0])
        for d, ax in self.dims.items():
            s[d] //= self.mesh.sizes[ax]
        return tuple(s)


class MPGatherOp(Op):
    """Shard -> replicated: all-gather along each split dim over its mesh axis."""

    def __init__(self, node, mesh, dims, ctx=None):
        super().__init__(MPGatherOp, [node], ctx)
        self.mesh, self.dims = mesh, dict(dims)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        r = _rank()
        for d, ax in self.dims.items():
            grp = self.mesh.group(r, (ax,))
            cm = _comm(grp)
            if cm is None:
                continue
            xt = x.movedim(d, 0).contiguous()
            out = torch.empty((xt.shape[0] * len(grp),) + tuple(xt.shape[1:]), dtype=xt.dtype, device=xt.device)
            cm.all_gather(out, xt)
            x = out.movedim(0, d)
        return x.contiguous()

    def gradient(self, output_grad):
        return [MPSliceOp(output_grad, self.mesh, self.dims, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        s = list(input_shapes[0])
        for d, ax in self.dims.items():
            s[d] *= self.mesh.sizes[ax]
        return tuple(s)


class MPReduceOp(Op):
    """Partial over ``axes`` -> replicated over them (all-reduce SUM); grad identity."""

    def __init__(self, node, mesh, axes, ctx=None):
        super().__init__(MPReduceOp, [node], ctx)
        self.mesh, self.axes = mesh, tuple(axes)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        x = input_vals[0]
        cm = _comm(self.mesh.group(_rank(), self.axes))
        if cm is None:
            return x
        y = x.clone()
        cm.all_reduce(y)
        return y

    def gradient(self, output_grad):
        return [output_grad]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


class MPCopyOp(Op):
    """Identity forward; backward all-reduces the gradient over ``axes`` (the
    operand is replicated over those axes but consumed by different shards)."""

    def __init__(self, node, mesh, axes, ctx=None):
        super().__init__(MPCopyOp, [node], ctx)
        self.mesh, self.axes = mesh, tuple(axes)

    def compute(self, input_vals, output_val=None, stream_handle=None):
        return input_vals[0]

    def gradient(self, output_grad):
        return [MPReduceOp(output_grad, self.mesh, self.axes, ctx=self.raw_ctx)]

    def infer_shape(self, input_shapes):
        return input_shapes[0]


# ---- the pass --------------------------------------------------------------------------
class _Status(object):
    """Distribution of a value: split dims {tensor_dim: mesh_axis} on a mesh."""

    def __init__(self, mesh=None, dims=None):
        self.mesh, self.dims = mesh, dict(dims or {})

    @property
    def replicated(self):
        return not self.dims

    def same(self, o):
        return (self.replicated and o.replicated) or (
            self.mesh is not None and o.mesh is not None and self.mesh.key() == o.mesh.key() and
            self.dims == o.dims)


def _in_region(node):
    rc = node.raw_ctx
    return isinstance(rc, DeviceGroup) and rc.is_mp


def lower_dispatch(roots, world=None):
    """Rewrite the forward graph in place.  Returns the meshes used (their
    sub-communicators must be created by ``create_groups`` on every rank)."""
    from ..ops.executor import find_topo_sort
    from ..ops.linalg import MatMulOp
    from ..ops.shape import BroadcastToOp
    from ..ops import basic as B
    from .dispatch import DispatchOp
    topo = find_topo_sort(roots)
    if not any(isinstance(n, DispatchOp) for n in topo):
        return []
    if world is None:
        world = max(dist_env()[1], 1)
    status: Dict[Op, _Status] = {}
    meshes = []
    replacement: Dict[Op, Op] = {}

    def val(n):
        return replacement.get(n, n)

    def st(n):
        return status.get(n, _Status())

    consumers = {}
    for n in topo:
        for i in n.inputs:
            consumers.setdefault(i, []).append(n)

    for n in topo:
        n.inputs = [val(i) for i in n.inputs]
        if isinstance(n, DispatchOp):
            src = n.inputs[0]
            parts = n.parts or {}
            if not _in_region(n):
                # exit dispatch (e.g. (1,1) on a single device): gather to replicated
                s = st(src)
                replacement[n] = MPGatherOp(src, s.mesh, s.dims, ctx=n.raw_ctx) if not s.replicated else src
                status[replacement[n]] = _Status()
                continue
            # resolved when the consuming matmul fixes the mesh; record request
            n._mp_parts = {d: p for d, p in parts.items() if p > 1}
            status[n] = _Status()
            continue
        if isinstance(n, MatMulOp) and any(isinstance(i, DispatchOp) for i in n.inputs):
            a, b = n.inputs
            ta, tb = n.matmul_attr_trans_A, n.matmul_attr_trans_B
            pa = getattr(a, '_mp_parts', {}) if isinstance(a, DispatchOp) else {}
            pb = getattr(b, '_mp_parts', {}) if isinstance(b, DispatchOp) else {}
            am, ak = (1, 0) if ta else (0, 1)
            bk, bn = (1, 0) if tb else (0, 1)
            pm, pn = pa.get(am, 1), pb.get(bn, 1)
            pka, pkb = pa.get(ak, 1), pb.get(bk, 1)
            if pka > 1 and pkb > 1 and pka != pkb:
                raise ValueError('matmul dispatch: K splits of A and B differ (%s vs %s)' % (pa, pb))
            pk = max(pka, pkb)
            mesh = Mesh({'m': pm, 'k': pk, 'n': pn})
            if mesh.P != world:
                raise ValueError('dispatch mesh %s needs %d ranks, job has %d' % (mesh.sizes, mesh.P, world))
            if all(m.key() != mesh.key() for m in meshes):
                meshes.append(mesh)
            c = n.raw_ctx
            A0 = a.inputs[0] if isinstance(a, DispatchOp) else a
            B0 = b.inputs[0] if isinstance(b, DispatchOp) else b
            adims = {d: ax for d, ax in ((am, 'm'), (ak, 'k')) if mesh.sizes[ax] > 1}
            bdims = {d: ax for d, ax in ((bk, 'k'), (bn, 'n')) if mesh.sizes[ax] > 1}
            As = _shard(A0, st(A0), mesh, adims, c)
            Bs = _shard(B0, st(B0), mesh, bdims, c)
            if mesh.sizes['n'] > 1:
                As = MPCopyOp(As, mesh, ('n',), ctx=c)
            if mesh.sizes['m'] > 1:
                Bs = MPCopyOp(Bs, mesh, ('m',), ctx=c)
            n.inputs = [As, Bs]
            out = n
            if mesh.sizes['k'] > 1:
                red = MPReduceOp(n, mesh, ('k',), ctx=c)
                replacement[n] = red
                out = red
            status[out] = _Status(mesh, {d: ax for d, ax in ((0, 'm'), (1, 'n')) if mesh.sizes[ax] > 1})
            continue
        ins = [st(i) for i in n.inputs]
        split = [s for s in ins if not s.replicated]
        if not split:
            # leaving a region without an explicit dispatch is handled here too
            continue
        if not _in_region(n):
            # replicated consumer of sharded values: gather them
            new = []
            for i, s in zip(n.inputs, ins):
                new.append(MPGatherOp(i, s.mesh, s.dims, ctx=i.raw_ctx) if not s.replicated else i)
            n.inputs = new
            continue
        if isinstance(n, BroadcastToOp):
            src, ref = n.inputs
            s_ref = st(ref)
            if st(src).replicated and not s_ref.replicated:
                # bias broadcast against a sharded output: slice the bias on the
                # trailing dims it shares with the output
                off = len(_shape_hint(ref)) - len(_shape_hint(src)) if _shape_hint(src) else 1
                dims = {d - off: ax for d, ax in s_ref.dims.items() if d - off >= 0}
                n.inputs = [_shard(src, _Status(), s_ref.mesh, dims, n.raw_ctx), ref]
            status[n] = s_ref
            continue
        ref = split[0]
        for s in split[1:]:
            if not s.same(ref):
                raise ValueError('op %s: inputs with different model-parallel splits' % n.name)
        for i, s in zip(n.inputs, ins):
            if s.replicated and len(n.inputs) > 1 and not isinstance(n, BroadcastToOp):
                raise ValueError('op %s mixes a replicated and a sharded operand; dispatch both' % n.name)
        status[n] = ref
    for m in meshes:
        if all(m.key() != x.key() for x in PENDING_MESHES):
            PENDING_MESHES.append(m)
    return meshes


def _shape_hint(n):
    return getattr(n, 'shape', None) or ()


def _shard(node, s, mesh, dims, ctx):
    if not dims:
        return node
    if s.replicated:
        return MPSliceOp(node, mesh, dims, ctx=ctx)
    if s.mesh.key() == mesh.key() and s.dims == dims:
        return node
    # re-distribution: gather then slice
    return MPSliceOp(MPGatherOp(node, s.mesh, s.dims, ctx=ctx), mesh, dims, ctx=ctx)


# ---- strategy helpers (reference ModelParallel4CNN / 4LM / OneWeirdTrick4CNN) -------------
def model_parallel_cnn(node_list, settings):
    """Dispatch every fully-connected weight column-wise over all workers."""
    return _dispatch_weights(node_list, axis=1)


def model_parallel_lm(node_list, settings):
    return _dispatch_weights(node_list, axis=1)


def one_weird_trick(node_list, settings):
    """Krizhevsky's 'one weird trick': data-parallel convolutions, model-parallel
    fully-connected layers -- here the FC weights are split column-wise while the
    rest stays replicated (DP handled by the DataParallel strategy)."""
    return _dispatch_weights(node_list, axis=1)


def _dispatch_weights(node_list, axis):
    from ..ops.executor import find_topo_sort
    from ..ops.linalg import MatMulOp
    from ..ops.variable import PlaceholderOp
    from .dispatch import DispatchOp
    world = max(dist_env()[1], 1)
    if world <= 1:
        return node_list
    dg = DeviceGroup([tuple('gpu:%d' % i for i in range(world))])
    for n in find_topo_sort(node_list):
        if isinstance(n, MatMulOp) and isinstance(n.inputs[1], PlaceholderOp) and n.inputs[1].trainable:
            w = n.inputs[1]
            if (w.shape or (0, 0))[axis] % world:
                continue
            d = DispatchOp(w, {axis: world}, ctx=dg)
            n.inputs[1] = d
            n.raw_ctx = dg
            a = n.inputs[0]
            if not isinstance(a, DispatchOp):
                n.inputs[0] = DispatchOp(a, {}, ctx=dg)
    return node_list
