"""CPU tests of the multi-rank agreement logic (no GPU): the start-up chain check's
store vote (VERDICT r3 #3a) and the xGMI grid-cap agreement for ranks spread unevenly over
GPUs."""
import threading

import pytest

from ddp_amd.engine.fused_step import agree
from ddp_amd.parallel.xgmi import check_blocks_agree, grid_cap_for, max_sharing


class FakeStore:
    """The two c10d store calls the code uses: set, and a blocking get."""

    def __init__(self):
        self.d, self.cv = {}, threading.Condition()

    def set(self, k, v):
        with self.cv:
            self.d[k] = v
            self.cv.notify_all()

    def get(self, k):
        with self.cv:
            assert self.cv.wait_for(lambda: k in self.d, timeout=10), k
            return self.d[k]


def _vote(oks):
    st, out = FakeStore(), [None] * len(oks)

    def rank(r):
        out[r] = agree(st, "k", r, len(oks), oks[r])

    th = [threading.Thread(target=rank, args=(r,)) for r in range(len(oks))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return out


@pytest.mark.parametrize("oks,want", [([True] * 4, True), ([True, True, False, True], False),
                                      ([False] * 3, False), ([True], True)])
def test_chain_vote_is_unanimous(oks, want):
    # one rank's mismatch downgrades EVERY rank (the same decision everywhere)
    assert _vote(oks) == [want] * len(oks)


def test_chain_vote_single_process():
    assert agree(None, "k", 0, 1, True) and not agree(None, "k", 0, 1, False)


def test_grid_cap_uneven_sharing_agrees():
    # world 3 on 2 GPUs: ranks 0 and 2 share GPU A, rank 1 is alone on GPU B
    bus = ["0000:05:00.0", "0000:15:00.0", "0000:05:00.0"]
    m = max_sharing(bus)
    assert m == 2
    caps = [grid_cap_for(256, m) for _ in range(3)]  # every rank computes from the same m
    assert len(set(caps)) == 1 and caps[0] == 32
    assert max_sharing(["a", "b", "c"]) == 1 and grid_cap_for(256, 1) == 256


def test_block_mismatch_fails_setup():
    check_blocks_agree([[32, 4], [32, 4], [32, 4]])
    with pytest.raises(RuntimeError):
        check_blocks_agree([[32, 4], [256, 4], [32, 4]])
