"""The counter protocol of the barrier-free tile experiment
(csrc/device/rt2_k5_dtiles.h, variants 269/270), simulated on the CPU: NW
waves as generators interleaved at random, random per-group costs, random
non-sweeping waves, segments of 1..8 tiles joined by the vote barrier.
Checks: no deadlock, no wave reads a tile before every wave's pieces of it
landed, no buffer is overwritten before every wave has read its previous
tile."""
import random
def run(NW, nt_list, seed, K=3, wait_for_readers=True):
    rnd = random.Random(seed)
    land = [0, 0]; done = [0, 0]
    # buffer contents: (tile id, set of waves whose pieces landed)
    buf = [None, None]
    reads_done = {}  # tile -> set of waves that finished reading
    log = []
    def wave(w):
        gbase = 0
        for nt in nt_list:           # segments (vote barrier between them)
            g0 = gbase; gbase += nt
            compute = rnd.random() < 0.8
            issued = 0; signalled = 0; fresh = False
            inflight = []  # tiles issued whose pieces not yet 'landed' (landing is instant at signal)
            def issue(t):
                g = g0 + t; b = g & 1
                # overwrite check: previous tile in buffer b must be read by all
                if g >= 2:
                    assert len(reads_done.get(g - 2, ())) == NW, ("overwrite", g, w)
                if buf[b] is None or buf[b][0] != g:
                    buf[b] = (g, set())
            def signal_land(t):
                g = g0 + t
                assert buf[g & 1][0] == g
                buf[g & 1][1].add(w); land[g & 1] += 1
            def read_by_all(g):
                return not wait_for_readers or done[g & 1] >= NW * (g // 2 + 1)
            issue(0); issued = 1
            if nt > 1: issue(1); issued = 2
            yield
            signal_land(0); signalled = 1
            if nt > 1: signal_land(1); signalled = 2
            for t in range(nt):
                g = g0 + t; b = g & 1
                while land[b] < NW * (g // 2 + 1):
                    yield
                assert buf[b][0] == g and len(buf[b][1]) == NW, ("read before landed", g)
                if compute:
                    for gi in range(K):
                        if t >= 1:
                            if signalled < issued and not fresh:
                                signal_land(signalled); signalled += 1
                            fresh = False
                            if issued == t + 1 and t + 1 < nt and read_by_all(g0 + t - 1):
                                issue(t + 1); issued += 1; fresh = True
                        for _ in range(rnd.choice([1, 1, 2, 5, 20])):
                            assert buf[b][0] == g, ("tile overwritten while reading", g)
                            yield
                reads_done.setdefault(g, set()).add(w); done[b] += 1
                if t + 1 < nt:
                    if issued == t + 1:
                        while not read_by_all(g - 1):
                            yield
                        issue(t + 1); issued += 1
                    if signalled == t + 1:
                        signal_land(t + 1); signalled += 1
                fresh = False
            yield ("barrier",)
    gens = [wave(w) for w in range(NW)]
    state = [None] * NW
    steps = 0
    seg = 0
    while True:
        active = [w for w in range(NW) if state[w] != "end" and state[w] != "barrier"]
        if not active:
            if all(s == "end" for s in state): return steps
            state = [None if s == "barrier" else s for s in state]; seg += 1
            continue
        w = rnd.choice(active)
        try:
            r = next(gens[w])
            if r == ("barrier",): state[w] = "barrier"
        except StopIteration:
            state[w] = "end"
        steps += 1
        if steps > 2_000_000: raise RuntimeError("deadlock?")


def test_tile_counter_protocol():
    for seed in range(120):
        NW = random.Random(seed).choice([2, 3, 12])
        nts = [random.Random(seed + 7 + k).choice([1, 2, 3, 5, 8]) for k in range(4)]
        run(NW, nts, seed)


def test_simulation_detects_a_missing_reader_wait():
    """Issuing a tile without waiting for every wave to have read its
    buffer's previous tile is caught (an overwrite while a wave reads)."""
    import pytest
    with pytest.raises(AssertionError):
        for seed in range(120):
            run(12, [5, 8, 3], seed, wait_for_readers=False)
