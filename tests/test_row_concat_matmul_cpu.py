"""RowConcatMatMulOp (the local experts' second GEMMs written as row blocks of one
output) against concatenate(matmul_i) on the CPU: forward and every gradient."""
import numpy as np

import hetu_61a7_amd as ht


def test_row_concat_matmul_matches_concat_of_matmuls():
    rng = np.random.RandomState(0)
    xs_v = [rng.randn(6, 5).astype(np.float32) for _ in range(3)]
    ws_v = [rng.randn(5, 4).astype(np.float32) for _ in range(3)]
    dy = rng.randn(18, 4).astype(np.float32)

    def run(fused):
        xs = [ht.Variable(name='x%d' % i) for i in range(3)]
        ws = [ht.Variable(name='w%d' % i) for i in range(3)]
        if fused:
            y = ht.row_concat_matmul_op(xs, ws)
        else:
            y = ht.concatenate_op([ht.matmul_op(x, w) for x, w in zip(xs, ws)], axis=0)
        g = ht.Variable(name='g')
        loss = ht.reduce_sum_op(ht.mul_op(y, g), [0, 1])
        grads = ht.gradients(loss, xs + ws)
        ex = ht.Executor([y] + grads, ctx=ht.cpu(0))
        fd = {**{x: v for x, v in zip(xs, xs_v)}, **{w: v for w, v in zip(ws, ws_v)}, g: dy}
        return ex.run(feed_dict=fd, convert_to_numpy_ret_vals=True)
    a, b = run(True), run(False)
    assert a[0].shape == (18, 4)
    for u, v in zip(a, b):
        np.testing.assert_allclose(u, v, rtol=1e-5, atol=1e-5)
