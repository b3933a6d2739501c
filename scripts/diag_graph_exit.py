"""Run the memory-pool test's MLP script under HETU_ALLOCATOR=torch (hipGraph auto mode)
in a child process and print its full stderr: the interpreter-exit path of a captured
torch graph."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from test_memory_pool_gpu import _SCRIPT  # noqa: E402

for alloc in ('torch', 'bfc'):
    env = dict(os.environ, PYTHONPATH=ROOT, HETU_ALLOCATOR=alloc)
    r = subprocess.run([sys.executable, '-c', _SCRIPT], env=env, capture_output=True, text=True, timeout=180)
    print('== HETU_ALLOCATOR=%s rc=%d' % (alloc, r.returncode))
    print(r.stdout[-500:])
    print(r.stderr[:4000])
