"""ResNet family.

* ``resnet50_imagenet`` etc.: ImageNet-shaped ResNet-18/34/50/101/152 (v1.5,
  stride on the 3x3 conv) -- the BASELINE config-2 model (the reference only
  ships a CIFAR-style ResNet, ``examples/cnn/models/ResNet.py:81-134``).
* ``resnet_cifar``: the reference's CIFAR-style ResNet (channels 16->128).

Written with plain Hetu ops (conv2d_op / batch_normalization_op / relu_op /
add_op); ``Optimizer.minimize`` fuses BN+ReLU and BN+add+ReLU automatically.
"""
from __future__ import annotations

from .. import ops as O
from .. import initializers as init


def conv2d(x, cin, cout, kernel=3, stride=1, padding=1, name=''):
    w = init.he_normal(shape=(cout, cin, kernel, kernel), name=name + '_weight')
    return O.conv2d_op(x, w, padding=padding, stride=stride)


def bn(x, c, name, relu=False, momentum=0.1, eps=1e-5):
    s = init.ones(shape=(c,), name=name + '_scale')
    b = init.zeros(shape=(c,), name=name + '_bias')
    y = O.batch_normalization_op(x, s, b, momentum=momentum, eps=eps)
    return O.relu_op(y) if relu else y


def bottleneck(x, cin, width, stride, name):
    cout = 4 * width
    shortcut = x
    y = bn(conv2d(x, cin, width, 1, 1, 0, name + '_conv1'), width, name + '_bn1', relu=True)
    y = bn(conv2d(y, width, width, 3, stride, 1, name + '_conv2'), width, name + '_bn2', relu=True)
    y = bn(conv2d(y, width, cout, 1, 1, 0, name + '_conv3'), cout, name + '_bn3')
    if stride != 1 or cin != cout:
        shortcut = bn(conv2d(x, cin, cout, 1, stride, 0, name + '_down'), cout, name + '_bnd')
    return O.relu_op(O.add_op(y, shortcut)), cout


def basic_block(x, cin, cout, stride, name):
    shortcut = x
    y = bn(conv2d(x, cin, cout, 3, stride, 1, name + '_conv1'), cout, name + '_bn1', relu=True)
    y = bn(conv2d(y, cout, cout, 3, 1, 1, name + '_conv2'), cout, name + '_bn2')
    if stride != 1 or cin != cout:
        shortcut = bn(conv2d(x, cin, cout, 1, stride, 0, name + '_down'), cout, name + '_bnd')
    return O.relu_op(O.add_op(y, shortcut)), cout


_CFG = {18: ('basic', [2, 2, 2, 2]), 34: ('basic', [3, 4, 6, 3]), 50: ('bottle', [3, 4, 6, 3]),
        101: ('bottle', [3, 4, 23, 3]), 152: ('bottle', [3, 8, 36, 3])}


def resnet_imagenet(x, y_, depth=50, num_classes=1000):
    """x: [N,3,224,224], y_: one-hot [N,num_classes]. Returns (loss, logits)."""
    kind, blocks = _CFG[depth]
    h = bn(conv2d(x, 3, 64, 7, 2, 3, 'stem'), 64, 'stem_bn', relu=True)
    h = O.max_pool2d_op(h, 3, 3, 1, 2)
    cin = 64
    for si, (n, width) in enumerate(zip(blocks, [64, 128, 256, 512])):
        for bi in range(n):
            stride = 2 if (bi == 0 and si > 0) else 1
            nm = 'layer%d_%d' % (si + 1, bi)
            if kind == 'bottle':
                h, cin = bottleneck(h, cin, width, stride, nm)
            else:
                h, cin = basic_block(h, cin, width, stride, nm)
    h = O.avg_pool2d_op(h, 7, 7, 0, 1)
    h = O.array_reshape_op(h, (-1, cin))
    w = init.he_normal(shape=(cin, num_classes), name='fc_weight')
    b = init.zeros(shape=(num_classes,), name='fc_bias')
    logits = O.linear_op(h, w, b)
    loss = O.reduce_mean_op(O.softmaxcrossentropy_op(logits, y_), [0])
    return loss, logits


def resnet50_imagenet(x, y_, num_classes=1000):
    return resnet_imagenet(x, y_, 50, num_classes)


def resnet_cifar(x, y_, depth=18, num_classes=10):
    """Reference-style CIFAR ResNet (examples/cnn/models/ResNet.py)."""
    kind, blocks = _CFG[depth]
    h = bn(conv2d(x, 3, 16, 3, 1, 1, 'conv0'), 16, 'bn0', relu=True)
    cin = 16
    widths = [16, 32, 64, 128] if kind == 'basic' else [16, 32, 64, 128]
    for si, (n, width) in enumerate(zip(blocks, widths)):
        for bi in range(n):
            stride = 2 if (bi == 0 and si > 0) else 1
            nm = 'res%d_%d' % (si, bi)
            if kind == 'bottle':
                h, cin = bottleneck(h, cin, width, stride, nm)
            else:
                h, cin = basic_block(h, cin, width, stride, nm)
    h = O.avg_pool2d_op(h, 4, 4, 0, 1)
    h = O.array_reshape_op(h, (-1, cin))
    w = init.he_normal(shape=(cin, num_classes), name='fc_weight')
    b = init.zeros(shape=(num_classes,), name='fc_bias')
    logits = O.linear_op(h, w, b)
    loss = O.reduce_mean_op(O.softmaxcrossentropy_op(logits, y_), [0])
    return loss, logits


def resnet18(x, y_, num_classes=10):
    return resnet_cifar(x, y_, 18, num_classes)


def resnet34(x, y_, num_classes=10):
    return resnet_cifar(x, y_, 34, num_classes)


def resnet50(x, y_, num_classes=10):
    return resnet_cifar(x, y_, 50, num_classes)
