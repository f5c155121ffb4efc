"""The tail-job protocol of the LDS-resident kernel (csrc/device/rt2_k5_resident.h,
MfmaSpec::tail_jobs), simulated on the CPU.

NW waves are generators interleaved at random, one LDS operation per step
(every load, store, compare-and-swap, atomic add / min is its own step, as on
the hardware).  Each wave traces a random number of segments; once it is in
the tail and helpers exist it posts some segments as jobs of nu = min(8,
helpers) units (random per-unit candidate hits) and waits for them; a wave
with nothing left helps (claims and serves units) until no wave is busy.  Checks, over many
seeds and wave counts:
  - every unit of every posted job is served exactly once, and the owner
    reads its keys only after all of them (its result = the minimum over all
    the job's units: what the one-wave sweep computes);
  - a unit is always served on the ray data of the epoch it was claimed for;
  - no deadlock: every wave finishes within a step bound;
  - helpers leave only when no wave is busy.
A mutant with the unit count and the next-unit counter in separate words
(reset one after the other) is caught serving a unit twice."""
import random

SLOTS = 6


class Board:
    def __init__(self, nw):
        self.ticket = [0] * SLOTS  # epoch << 8 | nu << 4 | next
        self.done = [0] * SLOTS
        self.owner = [0] * SLOTS
        self.busy = nw
        self.key = [[None] * 4 for _ in range(SLOTS)]
        self.data_epoch = [0] * SLOTS  # epoch whose rays are in the slot
        self.cands = [None] * SLOTS   # per unit candidate lists (what the rays would hit), per slot
        # split mutant
        self.nu = [0] * SLOTS
        self.next = [0] * SLOTS


def claim(b, j, split):
    """lane 0's claim loop: yields between LDS operations; returns (u, nu, epoch) or None."""
    if split:
        nu = b.nu[j]
        yield
        u = b.next[j]
        b.next[j] += 1  # atomic add (one step)
        yield
        return (u, nu, b.data_epoch[j]) if u < nu else None
    t = b.ticket[j]
    yield
    while (t & 15) < ((t >> 4) & 15):
        cur = b.ticket[j]  # compare-and-swap: one step
        if cur == t:
            b.ticket[j] = t + 1
            yield
            return (t & 15, (t >> 4) & 15, t >> 8)
        t = cur
        yield
    return None


def serve(b, j, u, nu, ep, served, log):
    # the unit reads the rays of its epoch
    assert b.data_epoch[j] == ep, ("stale rays", j, u, ep, b.data_epoch[j])
    yield
    key = (j, ep, u)
    assert key not in served, ("unit served twice", key)
    served.add(key)
    for r, c in enumerate(b.cands[j][u]):
        if c is not None:
            old = b.key[j][r]
            b.key[j][r] = c if old is None else min(old, c)  # atomic min: one step
            yield
    b.done[j] += 1  # atomic add, release
    yield


def wave(w, b, rnd, nw, split, served, log, jobs_done):
    nseg = rnd.randint(0, 6)
    tail_from = rnd.randint(0, nseg)
    slot = -1
    epoch = 0
    for seg in range(nseg):
        yield
        helpers = nw - b.busy
        if seg >= tail_from and helpers > 0 and rnd.random() < 0.8:
            if slot < 0:
                for j in range(SLOTS):
                    if b.owner[j] == 0:  # compare-and-swap
                        b.owner[j] = w + 1
                        slot = j
                        yield
                        break
                    yield
                if slot >= 0:
                    epoch = b.ticket[slot] >> 8
            if slot >= 0:
                j = slot
                nu = min(8, helpers)
                # the rays and the keys, then the ticket (release)
                b.data_epoch[j] = -1  # writing
                yield
                cands = [[(rnd.random() if rnd.random() < 0.5 else None) for _ in range(4)] for _ in range(nu)]
                b.cands[j] = cands
                b.key[j] = [None] * 4
                epoch = (epoch + 1) & 0xFFFFFF
                b.data_epoch[j] = epoch
                yield
                b.done[j] = 0
                yield
                if split:
                    b.nu[j] = nu  # mutant: two words, stored one after the other
                    yield
                    b.next[j] = 0
                else:
                    b.ticket[j] = epoch << 8 | nu << 4
                yield
                while b.done[j] < nu:  # the helpers serve the units
                    yield
                want = [min([c[r] for c in cands if c[r] is not None], default=None) for r in range(4)]
                assert b.key[j] == want, ("keys read before every unit was folded in", b.key[j], want)
                jobs_done.append((w, j, epoch, nu))
    # done: release the slot, leave the busy set, help
    if slot >= 0:
        b.owner[slot] = 0
        yield
    b.busy -= 1
    yield
    while True:
        served_one = False
        for j in range(SLOTS):
            c = yield from claim(b, j, split)
            if c is not None:
                yield from serve(b, j, c[0], c[1], c[2], served, log)
                served_one = True
        if not served_one:
            if b.busy == 0:
                return
            yield


def run(nw, seed, split=False, bound=200000):
    rnd = random.Random(seed)
    b = Board(nw)
    served, log, jobs_done = set(), [], []
    gens = [wave(w, b, random.Random(seed * 131 + w), nw, split, served, log, jobs_done) for w in range(nw)]
    alive = list(range(nw))
    steps = 0
    while alive:
        steps += 1
        assert steps < bound, "deadlock: waves still running"
        w = rnd.choice(alive)
        try:
            next(gens[w])
        except StopIteration:
            alive.remove(w)
    # every posted job's units were served exactly once
    for (w, j, ep, nu) in jobs_done:
        for u in range(nu):
            assert (j, ep, u) in served
    return len(jobs_done)


def test_tail_job_protocol_random_interleavings():
    jobs = 0
    for nw in (2, 3, 12, 16):
        for seed in range(120):
            jobs += run(nw, seed)
    assert jobs > 500  # the runs did post jobs


def test_split_ticket_mutant_is_caught():
    """Unit count and next-unit counter as two words reset one after the other:
    a helper between the two stores claims a unit of the new job that is then
    handed out again."""
    caught = 0
    for nw in (3, 12, 16):
        for seed in range(200):
            try:
                run(nw, seed, split=True)
            except AssertionError as e:
                caught += 1
                assert "twice" in str(e) or "stale" in str(e) or "keys" in str(e) or "deadlock" in str(e)
    assert caught > 0
