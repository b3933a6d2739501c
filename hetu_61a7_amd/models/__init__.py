"""Model zoo (reference examples/{cnn,ctr,nlp,moe,gnn,rec}/models)."""
from .resnet import resnet_imagenet, resnet50_imagenet, resnet_cifar, resnet18, resnet34, resnet50
from .cnn import logreg, mlp, cnn_3_layers, lenet, alexnet, vgg16, vgg19, rnn, lstm
from .gcn import gcn, dist_gcn_15d
from .ncf import neural_mf
from .transformer import Transformer, TransformerConfig
