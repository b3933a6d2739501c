"""Operator library: the public factory names of reference ``gpu_ops/__init__.py``."""
from .node import Op, OutputSelectOp, select_output
from .variable import Variable, placeholder_op, PlaceholderOp
from .basic import *  # noqa: F401,F403
from .basic import (abs_op, abs_gradient_op, opposite_op, exp_op, log_op, log_grad_op, floor_op,
                    sqrt_op, rsqrt_op, sin_op, cos_op, tanh_op, tanh_gradient_op, sigmoid_op,
                    relu_op, relu_gradient_op, leaky_relu_op, leaky_relu_gradient_op, gelu_op,
                    gelu_gradient_op, pow_op, pow_gradient_op, const_pow_op, const_pow_gradient_op,
                    clamp_op, bool_op, masked_fill_op, one_hot_op, where_op, where_const_op, add_op,
                    addbyconst_op, minus_op, minus_byconst_op, mul_op, mul_byconst_op, div_op,
                    div_const_op, matrix_dot_op, max_op, min_op, oneslike_op, zeroslike_op,
                    full_op, full_like_op, rand_op, arange_op, reduce_to_shape_op)
from .shape import (array_reshape_op, array_reshape_gradient_op, transpose_op, broadcastto_op,
                    broadcast_shape_op, slice_op, slice_gradient_op, slice_assign_op,
                    slice_assign_matrix_op, slice_by_matrix_op, slice_by_matrix_gradient_op,
                    split_op, split_gradient_op, concat_op, concat_gradient_op, concatenate_op,
                    concatenate_gradient_op, pad_op, pad_gradient_op, repeat_op,
                    repeat_gradient_op, roll_op, interpolate_op, interpolate_grad_op, gather_op,
                    gather_gradient_op, indexing_op, indexing_grad_op, scatter_op, scatter1d_op,
                    scatter1d_grad_op, conv2d_broadcastto_op, conv2d_reducesum_op)
from .reduce import (reduce_sum_op, reduce_mean_op, reducesumaxiszero_op, sum_op, norm_op,
                     norm_gradient_op, argmax_op, argsort_op, topk_idx_op, topk_val_op,
                     cumsum_with_bias_op)
from .linalg import (matmul_op, matmul_act_dropout_op, row_concat_matmul_op, RowConcatMatMulOp, linear_op, addmm_op, addmm_gradient_op, baddbmm_op,
                     batch_matmul_op, csrmv_op, csrmm_op)
from .nn import (conv2d_op, conv2d_gradient_of_data_op, conv2d_gradient_of_filter_op,
                 conv2d_add_bias_op, avg_pool2d_op, avg_pool2d_gradient_op, max_pool2d_op,
                 max_pool2d_gradient_op, batch_normalization_op, batch_normalization_gradient_op,
                 batch_normalization_gradient_of_data_op, batch_normalization_gradient_of_scale_op,
                 batch_normalization_gradient_of_bias_op, fused_bn_relu_op, fused_bn_add_relu_op,
                 layer_normalization_op, layer_normalization_gradient_op, dropout_add_layernorm_op,
                 layer_normalization_gradient_of_data_op, layer_normalization_gradient_of_scale_op,
                 layer_normalization_gradient_of_bias_op, instance_normalization2d_op,
                 instance_normalization2d_gradient_op, dropout_op, dropout_gradient_op,
                 dropout_gradient_recompute_op, dropout2d_op, dropout2d_gradient_op, AuxResult)
from .loss import (softmax_func, softmax_op, softmax_gradient_op, softmaxcrossentropy_op,
                   softmaxcrossentropy_gradient_op, softmaxcrossentropy_sparse_op,
                   softmaxcrossentropy_sparse_gradient_op, crossentropy_op,
                   crossentropy_gradient_op, crossentropy_sparse_op,
                   crossentropy_sparse_gradient_op, binarycrossentropy_op,
                   binarycrossentropy_gradient_op, nll_loss_op, nll_loss_grad_op)
from .embedding import embedding_lookup_op, embedding_lookup_gradient_op
from .transfer import datah2d_op, datad2h_op, datah2d_sparse_op, datad2h_sparse_op
from .comm import (allreduceCommunicate_op, allreduceCommunicatep2p_op,
                   groupallreduceCommunicate_op, allgatherCommunicate_op,
                   reducescatterCommunicate_op, broadcastCommunicate_op, reduceCommunicate_op,
                   alltoall_op, halltoall_op, pipeline_send_op, pipeline_receive_op)
from .moe import (layout_transform_op, layout_transform_gradient_op, reverse_layout_transform_op,
                  reverse_layout_transform_gradient_data_op,
                  reverse_layout_transform_gradient_gate_op, reverse_layout_transform_no_gate_op,
                  reverse_layout_transform_no_gate_gradient_op, balance_assignment_op,
                  sam_group_sum_op, sam_max_op, sammax_grad_op, group_topk_idx_op, topk_gating_op,
                  topk_locations_op)
from .ps_ops import (parameterServerCommunicate_op, parameterServerSparsePull_op,
                     ParameterServerCommunicateOp, ParameterServerSparsePullOp)
from .executor import Executor, HetuConfig, gradients, find_topo_sort
from .attention import attention_op, AttentionOp, AttentionGradientOp, packed_attention_op
from .distgcn import distgcn_15d_op, DistGCN_15dOp, make_15d_groups, partition_15d
from .mlm import masked_positions_op, take_rows_op, MaskedPositionsOp, TakeRowsOp, PutRowsOp
