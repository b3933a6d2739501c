"""Elastic recovery: heturun --max-restarts relaunches a failed
2-worker DP group; the workers resume from the last atomically committed
snapshot (weights + momentum state + step counter) and finish with exactly
the parameters of an uninterrupted run.  Fault injection: rank 1 exits with
status 3 after step 7 on the first attempt only (HETU_RESTART_COUNT=0)."""
import os
import subprocess
import sys
import textwrap

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

JOB = textwrap.dedent('''
    import os, sys
    import numpy as np
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.utils import checkpoint
    from hetu_61a7_amd.parallel import comm
    ckpt, out, crash_at = sys.argv[1], sys.argv[2], int(sys.argv[3])
    zero = len(sys.argv) > 4 and sys.argv[4] == 'zero'
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    attempt = int(os.environ.get('HETU_RESTART_COUNT', '0'))
    rng = np.random.RandomState(5)
    x, y_ = ht.Variable(name='x'), ht.Variable(name='y_')
    W1 = ht.Variable(name='w1', value=(rng.randn(12, 16) * 0.3).astype(np.float32))
    W2 = ht.Variable(name='w2', value=(rng.randn(16, 3) * 0.3).astype(np.float32))
    loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(
        ht.matmul_op(ht.relu_op(ht.matmul_op(x, W1)), W2), y_), [0])
    adam = len(sys.argv) > 4 and sys.argv[4] == 'adam'
    if zero:   # ZeRO-1: every rank owns half of the Adam moments
        train = ht.optim.AdamOptimizer(0.01).minimize(loss)
        ex = ht.Executor({'train': [loss, train]}, dist_strategy=ht.dist.DataParallel('allreduce'),
                         zero=1, bucket_mb=0.001)
        assert train.zero
    elif adam:
        train = ht.optim.AdamOptimizer(0.01).minimize(loss)
        ex = ht.Executor({'train': [loss, train]}, dist_strategy=ht.dist.DataParallel('allreduce'),
                         bucket_mb=0.001)
    else:
        train = ht.optim.MomentumOptimizer(0.05, 0.9).minimize(loss)
        ex = ht.Executor({'train': [loss, train]}, dist_strategy=ht.dist.DataParallel('allreduce'))
    start = checkpoint.resume(ex, ckpt)
    for step in range(start, 10):
        r = np.random.RandomState(1000 + step * world + rank)   # data keyed by (step, rank)
        X = r.randn(8, 12).astype(np.float32)
        Y = np.eye(3, dtype=np.float32)[r.randint(0, 3, 8)]
        ex.run('train', feed_dict={x: X, y_: Y})
        if (step + 1) % 3 == 0:
            checkpoint.save_resumable(ex, ckpt, step + 1)
        if attempt == 0 and rank == 1 and step + 1 == crash_at:
            if len(sys.argv) > 4 and sys.argv[4] == 'watchdog':
                # an RCCL async error surfaces while this rank is parked in a collective:
                # the watchdog thread (not the training loop) must end the process
                from hetu_61a7_amd.parallel import watchdog
                import time

                class FakeComm(object):
                    def async_error(self):
                        return 6          # ncclRemoteError
                    def abort(self):
                        sys.stderr.write('fake comm aborted\\n')
                    def __repr__(self):
                        return 'FakeComm'
                fake = FakeComm()
                watchdog.get().register(fake)
                time.sleep(120)           # "stuck": only the watchdog can end this
            os._exit(3)
    if rank == 0:
        np.savez(out, start=start, **checkpoint.state_dict(ex))
    comm.destroy()
''')


def _run(tmp_path, tag, crash_at, restarts, extra=(), env_extra=None):
    script = tmp_path / 'job.py'
    script.write_text(JOB)
    ckpt, out = tmp_path / ('ckpt_' + tag), tmp_path / (tag + '.npz')
    env = dict(os.environ, PYTHONPATH=ROOT, HETU_USE_CONFIG='0', **(env_extra or {}))
    env.pop('MASTER_PORT', None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bin', 'heturun'), '-w', '2',
                        '--max-restarts', str(restarts), sys.executable, str(script),
                        str(ckpt), str(out), str(crash_at)] + list(extra),
                       env=env, capture_output=True, text=True, timeout=240)
    return r, out, ckpt


def test_restart_resumes_from_last_snapshot(tmp_path):
    ref, ref_out, _ = _run(tmp_path, 'ref', crash_at=-1, restarts=0)
    assert ref.returncode == 0, ref.stderr[-2000:]
    r, out, ckpt = _run(tmp_path, 'elastic', crash_at=7, restarts=2)
    assert r.returncode == 0, r.stderr[-2000:]
    assert 'restart 1/2' in r.stderr
    a, b = np.load(ref_out), np.load(out)
    assert int(a['start']) == 0 and int(b['start']) == 6   # resumed after step 6's snapshot
    for k in ('w1', 'w2'):
        np.testing.assert_allclose(b[k], a[k], rtol=1e-5, atol=1e-6)
    # keep=2: only the two newest snapshots survive, `latest` names the last one
    assert sorted(os.listdir(ckpt)) == ['latest', 'step_6', 'step_9']


def test_watchdog_async_error_restarts_group(tmp_path):
    """SURVEY §5.3 RCCL watchdog: an asynchronous communicator error on rank 1 (a fake
    communicator registered with the process's watchdog) ends that worker with the
    watchdog's exit code while its main thread is blocked; heturun relaunches the group,
    which resumes from the last snapshot and ends with the uninterrupted parameters."""
    ref, ref_out, _ = _run(tmp_path, 'wref', crash_at=-1, restarts=0)
    assert ref.returncode == 0, ref.stderr[-2000:]
    r, out, _ = _run(tmp_path, 'wd', crash_at=7, restarts=1, extra=['watchdog'],
                     env_extra={'HETU_WATCHDOG_POLL': '0.05'})
    assert r.returncode == 0, r.stderr[-3000:]
    assert 'hetu watchdog (rank 1): RCCL asynchronous error 6 on FakeComm' in r.stderr, r.stderr[-3000:]
    assert 'fake comm aborted' in r.stderr
    assert 'rc=75' in r.stderr and 'restart 1/1' in r.stderr
    a, b = np.load(ref_out), np.load(out)
    assert int(b['start']) == 6
    for k in ('w1', 'w2'):
        np.testing.assert_allclose(b[k], a[k], rtol=1e-5, atol=1e-6)


def test_no_restart_propagates_failure(tmp_path):
    r, _, _ = _run(tmp_path, 'fail', crash_at=4, restarts=0)
    assert r.returncode == 3


def test_zero1_restart_restores_every_rank_shard(tmp_path):
    """ZeRO-1 + Adam: each rank's 1/P moment shard is written to its own
    ``.ext.rank<r>`` file and read back by that rank, so the resumed run ends
    exactly where the uninterrupted one does (a rank restored from another
    rank's shard would drift)."""
    ref, ref_out, _ = _run(tmp_path, 'zref', crash_at=-1, restarts=0, extra=['zero'])
    assert ref.returncode == 0, ref.stderr[-2000:]
    r, out, ckpt = _run(tmp_path, 'zel', crash_at=7, restarts=1, extra=['zero'])
    assert r.returncode == 0, r.stderr[-2000:]
    a, b = np.load(ref_out), np.load(out)
    assert int(b['start']) == 6
    for k in ('w1', 'w2'):
        np.testing.assert_allclose(b[k], a[k], rtol=1e-5, atol=1e-6)
    snap = os.listdir(os.path.join(ckpt, 'step_9'))
    assert 'checkpoint.pkl.ext.rank0' in snap and 'checkpoint.pkl.ext.rank1' in snap


def test_zero1_resume_refuses_missing_rank_shard(tmp_path):
    """A ZeRO-1 resume whose rank shard is gone must fail loudly instead of
    continuing with zeroed Adam moments under the restored step count."""
    ref, _, ckpt = _run(tmp_path, 'zmiss', crash_at=-1, restarts=0, extra=['zero'])
    assert ref.returncode == 0, ref.stderr[-2000:]
    os.remove(os.path.join(ckpt, 'step_9', 'checkpoint.pkl.ext.rank1'))
    r, _, _ = _run(tmp_path, 'zmiss', crash_at=-1, restarts=0, extra=['zero'])
    assert r.returncode != 0
    assert 'ZeRO-1 optimizer shard' in r.stderr


def test_zero1_resumes_from_a_non_zero_checkpoint(tmp_path):
    """A checkpoint written without ZeRO carries the full Adam moments: a ZeRO-1 run
    resumes from it by taking each rank's owned range of every bucket, and ends where
    the uninterrupted non-ZeRO run does."""
    ref, ref_out, ckpt = _run(tmp_path, 'adam', crash_at=-1, restarts=0, extra=['adam'])
    assert ref.returncode == 0, ref.stderr[-2000:]
    import shutil
    z = tmp_path / 'ckpt_zfrom'
    shutil.copytree(ckpt, z)
    # drop the last snapshot so the ZeRO run resumes at step 6 and trains 4 steps itself
    snaps = sorted(d for d in os.listdir(z) if d.startswith('step_'))
    for d in snaps:
        if d == 'step_9':
            shutil.rmtree(z / d)
    (z / 'latest').write_text('step_6\n')
    r, out, _ = _run(tmp_path, 'zfrom', crash_at=-1, restarts=0, extra=['zero'])
    assert r.returncode == 0, r.stderr[-2000:]
    a, b = np.load(ref_out), np.load(out)
    assert int(b['start']) == 6
    for k in ('w1', 'w2'):
        np.testing.assert_allclose(b[k], a[k], rtol=2e-5, atol=2e-6)


def test_sparse_update_torch_path_skips_untouched_rows():
    """optimizer.py's dense de-duplication marks untouched rows with id -1; the
    torch fallback of kernels.optim.sparse_update must not update table[-1]."""
    import torch
    from hetu_61a7_amd.kernels import optim as KO
    table = torch.ones(4, 3)
    s1 = torch.zeros(4, 3)
    ids = torch.tensor([0, -1, 2, -1])
    g = torch.ones(4, 3)
    KO.sparse_update('momentum', table, ids, g, s1=s1, lr=0.5, mu=0.9)
    np.testing.assert_allclose(table[:, 0].numpy(), [0.5, 1.0, 0.5, 1.0])
    np.testing.assert_allclose(s1[3].numpy(), 0.0)
