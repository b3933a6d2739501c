"""The examples/ entry points (reference examples/*) run end to end on the CPU
backend with tiny settings."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RUNS = [
    ['examples/cnn/main.py', '--model', 'mlp', '--dataset', 'cifar10', '--gpu', '-1', '--num-epochs', '1',
     '--max-steps', '3', '--synthetic', '--validate', '--timing'],
    ['examples/cnn/main.py', '--model', 'lenet', '--dataset', 'mnist', '--gpu', '-1', '--num-epochs', '1',
     '--max-steps', '2', '--synthetic', '--opt', 'adam', '--learning-rate', '0.001'],
    ['examples/cnn/main.py', '--model', 'lstm', '--dataset', 'mnist', '--gpu', '-1', '--num-epochs', '1',
     '--max-steps', '2', '--synthetic', '--opt', 'momentum'],
    ['examples/ctr/run_hetu.py', '--model', 'wdl_criteo', '--gpu', '-1', '--nepoch', '1', '--steps', '3', '--val'],
    ['examples/ctr/run_hetu.py', '--model', 'dfm_criteo', '--gpu', '-1', '--nepoch', '1', '--steps', '3'],
    ['examples/nlp/train_hetu_bert.py', '--gpu', '-1', '--hidden_size', '64', '--num_hidden_layers', '2',
     '--num_attention_heads', '2', '--seq_length', '32', '--train_batch_size', '4', '--vocab_size', '2000',
     '--steps', '2', '--fp32'],
    ['examples/moe/test_moe.py', '--gpu', '-1', '--batch_size', '2', '--num_tokens', '32', '--model_dim', '16',
     '--hidden_size', '32', '--num_steps', '2', '--gate', 'top'],
    ['examples/moe/test_moe_sam.py', '--gpu', '-1', '--batch_size', '2', '--num_tokens', '32', '--model_dim', '16',
     '--hidden_size', '32', '--num_steps', '2'],
    ['bin/heturun', '-w', '2', '-s', '1', sys.executable, 'examples/nlp/bert/train_hetu_bert_ps.py', '--gpu', '-1',
     '--hidden_size', '64', '--num_hidden_layers', '2', '--num_attention_heads', '2', '--seq_length', '32',
     '--train_batch_size', '4', '--vocab_size', '2000', '--steps', '2', '--fp32'],
    ['examples/gnn/run_single.py', '--gpu', '-1', '--nodes', '500', '--epochs', '2'],
    ['bin/heturun', '-w', '2', '-s', '1', sys.executable, 'examples/gnn/run_dist.py', '--cpu', '--num_epoch', '1',
     '--nodes', '2000', '--batch_size', '64', '--steps', '3'],
    ['bin/heturun', '-w', '2', '-s', '1', sys.executable, 'examples/gnn/run_dist_hybrid.py', '--cpu', '--num_epoch',
     '1', '--nodes', '2000', '--batch_size', '64', '--steps', '3', '--cache', 'lfuopt'],
    ['examples/rec/run_hetu.py', '--gpu', '-1', '--nepoch', '1', '--steps', '3', '--batch-size', '256', '--val'],
    ['examples/nlp/train_hetu_transformer.py', '--gpu', '-1', '--vocab_size', '200', '--d_model', '32', '--d_ff',
     '64', '--num_blocks', '1', '--num_heads', '4', '--maxlen1', '8', '--maxlen2', '9', '--batch_size', '4',
     '--steps', '2'],
    ['examples/runner/run_mlp.py', '--gpu', '-1', '--steps', '5'],
    ['examples/runner/run_wdl.py', '--config', 'local', '--nepoch', '2', '--val'],
    ['bin/heturun', '-w', '2', '-s', '1', sys.executable, 'examples/runner/run_wdl.py', '--config', 'lhy', '--cache',
     'lfuopt', '--nepoch', '1', '--val'],
    ['bin/heturun', '-w', '2', sys.executable, 'examples/runner/run_mlp.py', '--comm-mode', 'AllReduce',
     '--steps', '5'],
]


@pytest.mark.parametrize('cmd', RUNS, ids=[' '.join(c[:3]) for c in RUNS])
def test_example_runs(cmd):
    r = subprocess.run([sys.executable] + cmd, cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]


def test_parallel_equivalence_examples(tmp_path):
    """examples/runner/parallel: pipeline (GPipe, 1F1B), data+pipeline, a
    model-parallel split, the hand-wired send/recv pipeline (complex_pipeline_mlp,
    SURVEY §2.3 S9) and HetPipe with replicated stages synced through the PS
    (S8) reproduce the single-process losses
    (validate_results)."""
    import subprocess
    d = os.path.join(ROOT, 'examples', 'runner', 'parallel')
    out = str(tmp_path / 'results')
    env = dict(os.environ, PYTHONPATH=ROOT)
    heturun = [sys.executable, os.path.join(ROOT, 'bin', 'heturun')]
    script = os.path.join(d, 'mlp_parallel.py')
    runs = [[sys.executable, script, '--mode', 'base', '--cpu'],
            heturun + ['-w', '2', sys.executable, script, '--mode', 'pp', '--schedule', 'gpipe'],
            heturun + ['-w', '3', sys.executable, script, '--mode', 'pp', '--schedule', 'pipedream_flush'],
            heturun + ['-w', '4', sys.executable, script, '--mode', 'dp_pp', '--replicas', '2'],
            heturun + ['-w', '2', sys.executable, script, '--mode', 'mp', '--split', 'right'],
            heturun + ['-w', '3', sys.executable, os.path.join(d, 'complex_pipeline_mlp.py')],
            heturun + ['-w', '4', '-s', '1', sys.executable, script, '--mode', 'dp_pp', '--replicas', '2',
                       '--schedule', 'hetpipe']]
    for cmd in runs:
        r = subprocess.run(cmd + ['--out', out, '--steps', '3'], env=env, cwd=ROOT, capture_output=True,
                           text=True, timeout=240)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    r = subprocess.run([sys.executable, os.path.join(d, 'validate_results.py'), out], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.count(' ok') == 6, r.stdout


def test_glue_finetune_learns():
    """examples/nlp/bert/test_glue_hetu_bert.py: the sequence-classification head
    fine-tunes (3-label MNLI-shaped batches whose label is marked in the tokens).
    Runs in a fresh process: initial weights follow seed + node id (reference
    semantics), so in a long-lived process they depend on the ops built before."""
    import re
    cmd = [sys.executable, 'examples/nlp/bert/test_glue_hetu_bert.py', '--gpu_id', '-1', '--hidden_size', '64',
           '--num_hidden_layers', '2', '-a', '2', '-s', '16', '--train_batch_size', '32', '--vocab_size', '1100',
           '-e', '6', '--batches', '20', '--lr', '1e-3', '--dropout_prob', '0', '--task_name', 'mnli']
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    accs = [float(a) for a in re.findall(r'Accuracy = ([0-9.]+)', r.stdout)]
    assert len(accs) == 120
    assert np.mean(accs[:5]) < 0.5 and np.mean(accs[-10:]) > 0.55, accs


def test_gnn_dataloader_two_deep_queue():
    """GNNDataLoaderOp.step keeps the reference's one-step lag (dataloader.py:180-183):
    the graph handed in now is the one trained on at the next step."""
    import hetu_61a7_amd as ht
    d = ht.GNNDataLoaderOp(lambda g: np.full((2, 1), g, np.float32))
    y = ht.reduce_sum_op(d, [0, 1])
    ex = ht.Executor([y], ctx=ht.cpu(0))
    ht.GNNDataLoaderOp.step(1)
    ht.GNNDataLoaderOp.step(1)
    seen = []
    for g in (2, 3, 4):
        ht.GNNDataLoaderOp.step(g)
        seen.append(float(np.asarray(ex.run(convert_to_numpy_ret_vals=True)[0]).reshape(-1)[0]))
    assert seen == [2.0, 4.0, 6.0], seen
