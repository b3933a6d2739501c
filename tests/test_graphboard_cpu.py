"""Graphboard (reference python/graphboard): DOT text, SVG page and HTTP serving."""
import urllib.request

import numpy as np

import hetu_61a7_amd as ht


def _graph():
    x = ht.Variable(name='x')
    W = ht.init.random_normal((4, 3), name='W')
    y = ht.relu_op(ht.matmul_op(x, W))
    loss = ht.reduce_mean_op(y, [0, 1])
    train = ht.optim.SGDOptimizer(0.1).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0))
    ex.run('train', feed_dict={x: np.ones((2, 4), np.float32)})
    return ex


def test_dot_and_html():
    ex = _graph()
    dot = ht.graphboard.to_dot(ex)
    assert dot.startswith('digraph') and '->' in dot and 'MatMulOp' in dot
    page = ht.graphboard.to_html(ex)
    assert '<svg' in page and 'OptimizerOp' in page
    pos = ht.graphboard.layout(ex.subexecutor['train'].topo_order)
    for n, (k, L) in pos.items():   # every edge goes down at least one layer
        for i in n.inputs:
            if i in pos:
                assert pos[i][1] < L


def test_http_server():
    ex = _graph()
    srv = ht.graphboard.show(ex, port=0)
    port = srv.server_address[1]
    body = urllib.request.urlopen('http://127.0.0.1:%d/' % port, timeout=10).read().decode()
    dot = urllib.request.urlopen('http://127.0.0.1:%d/graph.dot' % port, timeout=10).read().decode()
    srv.shutdown()
    assert '<svg' in body and dot.startswith('digraph')
