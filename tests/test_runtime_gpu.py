"""Framework-owned HIP streams / events / copies (csrc/runtime/device_api.cc,
hetu_61a7_amd/runtime.py; reference src/cuda_common/gpu_runtime.cc:61-118)."""
import pytest
import torch

from hetu_61a7_amd import runtime as RT
from hetu_61a7_amd import kernels as K
from hetu_61a7_amd.kernels import elementwise as KE

pytestmark = pytest.mark.gpu


def test_stream_event_ordering_and_timing():
    s = RT.DeviceStream(priority=-1)
    x = torch.randn(1 << 22, device='cuda')
    start = RT.DeviceEvent(timing=True).record(s)
    s.wait_stream(torch.cuda.current_stream())          # x is ready before s runs
    with RT.use_stream(s):                               # the framework's current stream
        assert K.stream_ptr() == s.handle                 # hand-written kernels launch on it
        assert torch.cuda.current_stream().cuda_stream == s.handle   # torch follows it
        y = KE.unary('mul_c', x, 3.0)
    assert K.stream_ptr() != s.handle
    end = RT.DeviceEvent(timing=True).record(s)
    end.wait(torch.cuda.current_stream())               # the current stream waits for y
    torch.testing.assert_close(y, x * 3.0)
    end.synchronize()
    assert end.query() and s.query()
    assert end.elapsed_time(start) <= 0.0 <= start.elapsed_time(end)


def test_async_copies_on_a_framework_stream():
    s = RT.DeviceStream()
    src = torch.arange(1 << 16, dtype=torch.float32).pin_memory()
    dev = torch.empty(1 << 16, device='cuda')
    back = torch.empty(1 << 16).pin_memory()
    RT.memcpy_async(dev.data_ptr(), src.data_ptr(), src.numel() * 4, 'h2d', s)
    RT.memcpy_async(back.data_ptr(), dev.data_ptr(), src.numel() * 4, 'd2h', s)
    s.synchronize()
    assert torch.equal(back, src)


def test_executor_streams_are_framework_streams():
    import hetu_61a7_amd as ht
    from hetu_61a7_amd.stream import Stream, Event
    st = Stream(ht.gpu(0))
    ev = Event(ht.gpu(0))
    assert st.native is not None and st.handle == st.native.handle
    with st:
        assert torch.cuda.current_stream().cuda_stream == st.handle
    ev.record(st)
    ev.sync()
