"""C1 (BASELINE.json configs[0]): the unpartitioned pattern at 10M ticks, 100
symbols, R = 1 ev/ms on the HIP path (sh_run_device, one key), bit-exact
against the oracle on a 200k-event prefix and against the vectorised
restatement (pinned to the oracle for C1 in tests/test_c2_checker.py) on the
full 10M."""
import numpy as np
import pytest

from c2_check import c2_expected
from oracle_engine import run_columns_oracle
from siddhi_amd import compiler, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _gpu(ts, k, p, v):
    import torch
    from siddhi_amd.device_run import DeviceRunner
    runner = DeviceRunner(compiler.compile_app(synth.C1_QUERY))
    dev = torch.device("cuda:0")
    zero = torch.zeros(len(ts), dtype=torch.int32, device=dev)
    cols = [torch.from_numpy(c).to(dev) for c in (k, p, v)]
    m, oseq, ovals = runner.run(torch.from_numpy(ts).to(dev), zero, cols, 1)
    torch.cuda.synchronize()
    r = (oseq.cpu().numpy(), ovals.cpu().numpy())
    runner.close()
    return r


def test_c1_prefix_vs_oracle():
    ts, k, p, v = synth.stock_stream(200_000, 100, 1, config_index=1)
    seq, _, vals, _ = run_columns_oracle(compiler.compile_app(synth.C1_QUERY), ts, [k, p, v], None)
    gseq, gvals = _gpu(ts, k, p, v)
    assert len(gseq) == len(seq) > 0
    assert np.array_equal(gseq, seq.astype(np.int64)) and np.array_equal(gvals, vals)


def test_c1_full_size_vs_restatement():
    ts, k, p, v = synth.stock_stream(10_000_000, 100, 1, config_index=1)
    eseq, evals = c2_expected(ts, k, p, v)
    gseq, gvals = _gpu(ts, k, p, v)
    assert len(gseq) == len(eseq) > 0
    assert np.array_equal(gseq, eseq) and np.array_equal(gvals, evals)
