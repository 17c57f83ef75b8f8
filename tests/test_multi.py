"""skv.multi.MultiCompactor: independent compactions dispatched to per-device workers (one ctx and
one host thread each, least-queued-bytes placement), results in submission order, errors carried
by each job's future. CPU test: workers built around the oracle; GPU test: two ctxs on GPU 0."""
import threading

import pytest

from skv import _abi, gen
from skv.multi import MultiCompactor

import pyoracle


class _OracleDev:
    def __init__(self, device):
        self.device = device
        self.thread = None
        self.jobs = 0

    def compact(self, streams, max_run_size, flags, with_info=False):
        self.thread = threading.get_ident()
        self.jobs += 1
        return pyoracle.compact(streams, max_run_size, flags, with_result=with_info)


def _jobs():
    jobs = [(gen.config2(seed=s, n_streams=4, n_records=300 + 50 * s, vsize=32, variant="B"), 16 << 10, 0)
            for s in range(10)]
    jobs.append(([(1, [b"\x02"])], 1 << 20, 0))  # a failing job: UnsupportedVersion
    return jobs


def test_multi_dispatch_with_oracle_workers():
    made = []

    def factory(d):
        c = _OracleDev(d)
        made.append(c)
        return c

    jobs = _jobs()
    with MultiCompactor([0, 1, 2], factory) as mc:
        futs = [mc.submit(*j) for j in jobs]
        for f, (streams, mx, fl) in zip(futs[:-1], jobs[:-1]):
            assert [r.data for r in f.result()] == [r.data for r in pyoracle.compact(streams, mx, fl)]
        with pytest.raises(_abi.RunError) as ei:
            futs[-1].result()
        assert ei.value.code == _abi.SKV_E_UNSUPPORTED_VERSION
    assert len(made) == 3 and sum(c.jobs for c in made) == len(jobs)
    assert all(c.jobs > 0 for c in made)  # the queue spread the work
    assert len({c.thread for c in made}) == 3  # one host thread per device ctx


@pytest.mark.gpu
def test_multi_two_ctxs_on_one_gpu():
    torch = pytest.importorskip("torch")
    torch.cuda.init()
    jobs = _jobs()
    with MultiCompactor([0, 0]) as mc:
        futs = [mc.submit(*j) for j in jobs]
        for f, (streams, mx, fl) in zip(futs[:-1], jobs[:-1]):
            assert [r.data for r in f.result()] == [r.data for r in pyoracle.compact(streams, mx, fl)]
        with pytest.raises(_abi.RunError):
            futs[-1].result()
