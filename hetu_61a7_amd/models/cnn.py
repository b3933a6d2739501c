"""Image-classification models of reference ``examples/cnn/models`` (LogReg,
MLP, CNN-3, LeNet, AlexNet, VGG16/19, RNN, LSTM); each returns (loss, logits)."""
from __future__ import annotations

from .. import ops as O
from .. import initializers as init


def _fc(x, shape, name, act=None):
    w = init.he_normal(shape=shape, name=name + '_weight')
    b = init.zeros(shape=shape[-1:], name=name + '_bias')
    return O.linear_op(x, w, b, activation=act)


def _loss(logits, y_):
    return O.reduce_mean_op(O.softmaxcrossentropy_op(logits, y_), [0])


def logreg(x, y_):
    """784 -> 10, zero init (reference LogReg.py)."""
    w = init.zeros((784, 10), name='logistic_regression_weight')
    b = init.zeros((10,), name='logistic_regression_bias')
    y = O.linear_op(x, w, b)
    return _loss(y, y_), y


def mlp(x, y_, in_dim=3072, hidden=(256, 256), num_classes=10):
    """Reference MLP: 3072 -> 256 -> 256 -> 10 with ReLU."""
    h = x
    d = in_dim
    for i, hd in enumerate(hidden):
        h = _fc(h, (d, hd), 'mlp_fc%d' % (i + 1), act='relu')
        d = hd
    y = _fc(h, (d, num_classes), 'mlp_fc%d' % (len(hidden) + 1))
    return _loss(y, y_), y


def _conv_relu(x, cin, cout, k, stride, pad, name):
    w = init.he_normal(shape=(cout, cin, k, k), name=name + '_weight')
    b = init.zeros(shape=(cout,), name=name + '_bias')
    return O.relu_op(O.conv2d_add_bias_op(x, w, b, padding=pad, stride=stride))


def cnn_3_layers(x, y_):
    x = O.array_reshape_op(x, (-1, 1, 28, 28))
    h = O.max_pool2d_op(_conv_relu(x, 1, 32, 5, 1, 2, 'cnn_conv1'), 2, 2, 0, 2)
    h = O.max_pool2d_op(_conv_relu(h, 32, 64, 5, 1, 2, 'cnn_conv2'), 2, 2, 0, 2)
    h = O.array_reshape_op(h, (-1, 7 * 7 * 64))
    y = _fc(h, (7 * 7 * 64, 10), 'cnn_fc')
    return _loss(y, y_), y


def lenet(x, y_):
    x = O.array_reshape_op(x, (-1, 1, 28, 28))
    h = O.max_pool2d_op(_conv_relu(x, 1, 6, 5, 1, 2, 'lenet_conv1'), 2, 2, 0, 2)
    h = O.max_pool2d_op(_conv_relu(h, 6, 16, 5, 1, 0, 'lenet_conv2'), 2, 2, 0, 2)
    h = O.array_reshape_op(h, (-1, 16 * 5 * 5))
    h = _fc(h, (400, 120), 'lenet_fc1', act='relu')
    h = _fc(h, (120, 84), 'lenet_fc2', act='relu')
    y = _fc(h, (84, 10), 'lenet_fc3')
    return _loss(y, y_), y


def alexnet(x, y_, num_classes=10):
    """CIFAR-sized AlexNet (reference AlexNet.py)."""
    h = O.max_pool2d_op(_conv_relu(x, 3, 64, 3, 1, 1, 'alex_conv1'), 2, 2, 0, 2)
    h = O.max_pool2d_op(_conv_relu(h, 64, 192, 3, 1, 1, 'alex_conv2'), 2, 2, 0, 2)
    h = _conv_relu(h, 192, 384, 3, 1, 1, 'alex_conv3')
    h = _conv_relu(h, 384, 256, 3, 1, 1, 'alex_conv4')
    h = O.max_pool2d_op(_conv_relu(h, 256, 256, 3, 1, 1, 'alex_conv5'), 2, 2, 0, 2)
    h = O.array_reshape_op(h, (-1, 256 * 4 * 4))
    h = O.dropout_op(_fc(h, (4096, 4096), 'alex_fc1', act='relu'), 0.5)
    h = O.dropout_op(_fc(h, (4096, 4096), 'alex_fc2', act='relu'), 0.5)
    y = _fc(h, (4096, num_classes), 'alex_fc3')
    return _loss(y, y_), y


def _vgg(x, y_, cfg, num_classes):
    h, cin, i = x, 3, 0
    for v in cfg:
        if v == 'M':
            h = O.max_pool2d_op(h, 2, 2, 0, 2)
        else:
            w = init.he_normal(shape=(v, cin, 3, 3), name='vgg_conv%d_weight' % i)
            h = O.conv2d_op(h, w, padding=1, stride=1)
            s = init.ones((v,), name='vgg_bn%d_scale' % i)
            b = init.zeros((v,), name='vgg_bn%d_bias' % i)
            h = O.relu_op(O.batch_normalization_op(h, s, b))
            cin, i = v, i + 1
    h = O.array_reshape_op(h, (-1, 512))
    h = _fc(h, (512, 4096), 'vgg_fc1', act='relu')
    h = _fc(h, (4096, 4096), 'vgg_fc2', act='relu')
    y = _fc(h, (4096, num_classes), 'vgg_fc3')
    return _loss(y, y_), y


def vgg16(x, y_, num_classes=10):
    return _vgg(x, y_, [64, 64, 'M', 128, 128, 'M', 256, 256, 256, 'M', 512, 512, 512, 'M',
                        512, 512, 512, 'M'], num_classes)


def vgg19(x, y_, num_classes=10):
    return _vgg(x, y_, [64, 64, 'M', 128, 128, 'M', 256, 256, 256, 256, 'M', 512, 512, 512, 512,
                        'M', 512, 512, 512, 512, 'M'], num_classes)


def rnn(x, y_, diminput=28, dimhidden=128, dimoutput=10, nsteps=28):
    """Elman RNN over rows of a 28x28 image (reference RNN.py)."""
    wx = init.random_normal((diminput, dimhidden), stddev=0.1, name='rnn_wx')
    wh = init.random_normal((dimhidden, dimhidden), stddev=0.1, name='rnn_wh')
    b = init.zeros((dimhidden,), name='rnn_b')
    h = None
    for t in range(nsteps):
        xt = O.slice_op(x, (0, t * diminput), (-1, diminput))
        a = O.linear_op(xt, wx, b)
        if h is not None:
            a = O.add_op(a, O.matmul_op(h, wh))
        h = O.tanh_op(a)
    y = _fc(h, (dimhidden, dimoutput), 'rnn_out')
    return _loss(y, y_), y


def lstm(x, y_, diminput=28, dimhidden=128, dimoutput=10, nsteps=28):
    """LSTM over rows of a 28x28 image (reference LSTM.py); gates fused in one GEMM."""
    wx = init.random_normal((diminput, 4 * dimhidden), stddev=0.1, name='lstm_wx')
    wh = init.random_normal((dimhidden, 4 * dimhidden), stddev=0.1, name='lstm_wh')
    b = init.zeros((4 * dimhidden,), name='lstm_b')
    h = c = None
    for t in range(nsteps):
        xt = O.slice_op(x, (0, t * diminput), (-1, diminput))
        z = O.linear_op(xt, wx, b)
        if h is not None:
            z = O.add_op(z, O.matmul_op(h, wh))
        gi = O.sigmoid_op(O.slice_op(z, (0, 0), (-1, dimhidden)))
        gf = O.sigmoid_op(O.slice_op(z, (0, dimhidden), (-1, dimhidden)))
        go = O.sigmoid_op(O.slice_op(z, (0, 2 * dimhidden), (-1, dimhidden)))
        gg = O.tanh_op(O.slice_op(z, (0, 3 * dimhidden), (-1, dimhidden)))
        c = O.mul_op(gi, gg) if c is None else O.add_op(O.mul_op(gf, c), O.mul_op(gi, gg))
        h = O.mul_op(go, O.tanh_op(c))
    y = _fc(h, (dimhidden, dimoutput), 'lstm_out')
    return _loss(y, y_), y


def logreg_bench(args, world, rank, local):
    """BASELINE config 1: logistic regression on MNIST-shaped data (784 -> 10, zero init,
    batch 128, SGD lr 0.01; reference examples/cnn/main.py:24-27,114-119 with --gpu -1) on
    the CPU executor -- the native C++/OpenMP backend (kernels.cpu_native).  A step is one
    forward + backward + SGD update; the batches cycle through a fixed synthetic set.

    Returns (step, samples_per_step, cfg, metric, finish); ``step.extra()`` reports the
    ATen compute ops one steady-state step issued (torch CPU profiler) and the native
    backend's fallback count, both expected to be 0."""
    import numpy as np
    import torch
    import hetu_61a7_amd as ht
    from ..kernels import cpu_native
    B = args.batch or 128
    x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
    loss, _ = logreg(x, y_)
    train = ht.optim.SGDOptimizer(learning_rate=0.01).minimize(loss)
    ex = ht.Executor({'train': [loss, train]}, ctx=ht.cpu(0))
    rng = np.random.RandomState(1234 + rank)
    nb = 16
    X = torch.from_numpy(rng.rand(nb, B, 784).astype(np.float32))
    Y = torch.from_numpy(np.eye(10, dtype=np.float32)[rng.randint(0, 10, (nb, B))])
    it = [0]

    def step():
        i = it[0] % nb
        it[0] += 1
        return ex.run('train', feed_dict={x: X[i], y_: Y[i]})

    def extra():
        cpu_native.reset_fallbacks()
        from torch.profiler import profile, ProfilerActivity
        with profile(activities=[ProfilerActivity.CPU]) as prof:
            step()
        # allocation / view / metadata ops move no data; anything else is ATen compute.
        # aten::to and aten::contiguous are dispatchers that return their input unchanged
        # when nothing has to move -- a real conversion or copy shows up as the
        # aten::_to_copy / aten::clone / aten::copy_ it calls, which are counted
        meta = ('empty', 'empty_strided', 'empty_like', 'view', 'reshape', 'as_strided', 'expand', 'permute',
                'transpose', 'select', 'slice', 'detach', 'alias', 'unsqueeze', 'squeeze', 'resolve', 'lift',
                'result_type', 'is_', 'size', 'stride', 'numel', 'contiguous', 't', 'flatten', 'unfold',
                '_unsafe_view', 'set_', 'to', 'narrow', 'broadcast_to')
        compute = sorted({e.key for e in prof.key_averages() if e.key.startswith('aten::') and
                          e.key[6:].lstrip('_') not in meta and not any(e.key[6:] == m for m in meta)})
        return {'aten_compute_ops_per_step': compute, 'native_cpu_fallbacks': dict(cpu_native.FALLBACKS),
                'cpu_backend': 'native' if cpu_native.enabled() else 'aten',
                'omp_threads': int(cpu_native.lib().hetu_cpu_num_threads())}
    step.extra = extra
    cfg = {'model': 'logreg MNIST (784->10)', 'global_batch': B, 'seq_len': None, 'parallelism': 'cpu',
           'optimizer': 'sgd', 'device': 'cpu'}
    return step, B, cfg, 'samples/sec logreg MNIST CPU', None
