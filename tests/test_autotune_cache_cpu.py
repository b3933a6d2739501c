"""Persisted autotune decisions (kernels/autotune.py save / load / HETU_AUTOTUNE_CACHE)."""
import torch

from hetu_61a7_amd.kernels import autotune as A


def test_saved_decisions_are_taken_without_measuring(tmp_path, monkeypatch):
    monkeypatch.setattr(A, '_decisions', {})
    monkeypatch.setattr(A, '_loaded', {})
    key = ((8192, 768), (768, 1), torch.bfloat16, 'nt', 3)
    A._decisions[key] = 'hip3'
    A._decisions[('other', 1)] = 'hip0'
    p = tmp_path / 'tune.json'
    A.save(str(p))
    A._decisions.clear()
    assert A.load(str(p)) == 2
    called = []
    cands = {'hip0': lambda: called.append('hip0'), 'hip3': lambda: called.append('hip3')}
    assert A.choose(key, cands) == 'hip3'
    assert not called                      # no candidate ran
    assert A._decisions[key] == 'hip3'
    # a cached name the call site no longer offers is ignored
    A._decisions.clear()
    assert A.choose(key, {'hip0': lambda: None}) == 'hip0'
