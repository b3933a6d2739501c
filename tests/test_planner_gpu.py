"""Galvatron hardware model calibrated on the MI355X (achieved bf16 GEMM rate)."""
import pytest

pytestmark = pytest.mark.gpu


def test_calibrate_on_device():
    from hetu_61a7_amd.parallel.galvatron import Hardware, plan_bert
    hw = Hardware.calibrate(gpus=8)
    assert 1e14 < hw.flops < 3e15, hw.flops       # between 100 TF and the dense bf16 peak
    plan = plan_bert(global_batch=512, hw=hw)
    assert plan.throughput > 0
