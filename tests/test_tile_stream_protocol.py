"""CPU model of the tile stream's LDS-counter protocol (rt2_k5_tiles.h
sweep_kt_flow, MfmaSpec::tile_flow; DESIGN.md "LDS record tiles", round 6).

NW waves walk the same stream of tiles (stream index s: tile s % nt, buffer
s % NB); per tile a wave runs upkeep(force) then waits until all NW shares of
tile s have landed (landed[b] >= NW * (s // NB + 1)), sweeps its gn groups
(upkeep(false, gi == K // 2) before each group's products), and releases the
buffer (rel[b] += 1).  upkeep publishes a pending share once it is two groups
old (or at once when forced) and issues the wave's next share once every wave
has released that tile's buffer (rel[b] == NW * (s // NB)).  A share's DMA
lands after a random delay; publishing waits for it (s_waitcnt vmcnt(0)).
Segments are nt consecutive stream indices separated by a workgroup vote
(barrier), as in render_mfma_k5t.

Random interleavings of the waves (one atomic step at a time) check the two
safety properties the kernel relies on and that every run terminates:
  - no wave reads a buffer before every share of its tile has landed there;
  - no share is written into a buffer while some wave may still read the
    buffer's previous tile (its release has not happened).
The model follows the kernel statement by statement; a mutant that issues
without the release check is caught."""
import random

import pytest


class Model:
    def __init__(self, nw, nb, k, ng, segments, seed, check_release=True):
        self.nw, self.nb, self.k, self.ng = nw, nb, k, ng
        self.nt = (ng + k - 1) // k
        self.segments = segments
        self.rng = random.Random(seed)
        self.check_release = check_release
        self.landed = [0] * nb
        self.rel = [0] * nb
        # buffer contents: per buffer, the set of (stream index, share) pieces present
        self.buf_tile = [[None] * nw for _ in range(nb)]
        self.reading = [set() for _ in range(nb)]  # waves currently reading each buffer
        self.inflight = []  # (land_time, wave, s)
        self.time = 0

    def issue_share(self, w, s):
        b = s % self.nb
        # a DMA into b while a wave still reads b's previous tile is a violation
        for r in self.reading[b]:
            assert self.waves[r]["cur"] == s, f"share of {s} written into buffer {b} while wave {r} reads it"
        self.inflight.append((self.time + self.rng.randint(1, 40), w, s))

    def land(self):
        keep = []
        for t, w, s in self.inflight:
            if t <= self.time:
                self.buf_tile[s % self.nb][w] = s
            else:
                keep.append((t, w, s))
        self.inflight = keep

    def wave_landed(self, w):
        return not any(iw == w for _, iw, _ in self.inflight)

    def run(self):
        nw, nb, k = self.nw, self.nb, self.k
        self.waves = [dict(next=0, next_issue=0, pend=-1, age=0, cur=None, prog=self.program(i)) for i in range(nw)]
        done = [False] * nw
        steps = 0
        while not all(done):
            steps += 1
            assert steps < 2_000_000, "no progress (deadlock)"
            self.time += 1
            self.land()
            w = self.rng.randrange(nw)
            if done[w]:
                continue
            try:
                next(self.waves[w]["prog"])
            except StopIteration:
                done[w] = True
        return steps

    def program(self, w):
        """One wave's walk over all segments (a generator: one atomic step per yield)."""
        nw, nb, k = self.nw, self.nb, self.k
        W = None

        def upkeep(force, try_issue):
            if W["pend"] >= 0 and (force or W["age"] >= 2):
                # s_waitcnt vmcnt(0): block until this wave's pieces have landed
                while not self.wave_landed(w):
                    yield
                self.landed[W["pend"] % nb] += 1
                W["pend"] = -1
                yield
            if W["pend"] < 0 and try_issue:
                s = W["next_issue"]
                ok = self.rel[s % nb] == nw * (s // nb)
                if ok or not self.check_release:
                    self.issue_share(w, s)
                    W["pend"], W["age"], W["next_issue"] = s, 0, s + 1
                yield

        for seg in range(self.segments):
            # the workgroup vote between segments (a barrier)
            self.barrier_arrive(w, seg)
            while not self.barrier_open(seg):
                yield
            W = self.waves[w]
            for t in range(self.nt):
                s = W["next"]
                W["next"] += 1
                b, gn = s % nb, min(k, self.ng - t * k)
                yield from upkeep(True, True)
                while self.landed[b] < nw * (s // nb + 1):
                    yield from upkeep(True, True)
                    yield
                # every share of tile s is in buffer b
                assert all(x == s for x in self.buf_tile[b]), f"wave {w} reads tile {s} before it landed"
                W["cur"] = s
                self.reading[b].add(w)
                for gi in range(gn):
                    W["age"] += 1
                    yield from upkeep(False, gi == k // 2)
                    assert all(x == s for x in self.buf_tile[b]), f"buffer {b} overwritten under wave {w}"
                    yield
                self.reading[b].discard(w)
                W["cur"] = None
                self.rel[b] += 1
                yield
        # kernel end: wait for a share still in flight (s_waitcnt vmcnt(0))
        while not self.wave_landed(w):
            yield

    # vote barrier
    def barrier_arrive(self, w, seg):
        if not hasattr(self, "arrived"):
            self.arrived = {}
        self.arrived.setdefault(seg, set()).add(w)

    def barrier_open(self, seg):
        return len(self.arrived.get(seg, ())) == self.nw


@pytest.mark.parametrize("nw,nb,k,ng,segments", [(16, 2, 19, 60, 3), (12, 2, 19, 19, 3), (4, 2, 3, 10, 4),
                                                  (8, 4, 2, 9, 3), (2, 2, 1, 1, 5), (6, 2, 4, 23, 2)])
def test_tile_stream_safe_and_terminates(nw, nb, k, ng, segments):
    for seed in range(30):
        Model(nw, nb, k, ng, segments, seed).run()


def test_tile_stream_mutant_without_release_check_is_caught():
    caught = 0
    for seed in range(20):
        try:
            Model(4, 2, 3, 10, 3, seed, check_release=False).run()
        except AssertionError:
            caught += 1
    assert caught > 0
