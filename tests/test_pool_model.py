"""A CPU model of the path-pool kernel's scheduling (traceTilePool, sail_trace.hip), step for step: slot and work
allocation by per-wave atomics, the refill-and-sweep loop, the class counts of swept and waiting records, the
placement of full class waves and promoted leftovers, and the gather by perm. Paths are abstract (a class per bounce
and a miss probability), and the atomics' order between waves is shuffled. The model checks what the GPU kernel relies
on: placement positions are distinct and below the shaded count, no slot is carried by two lanes, every waiting record
is counted exactly once, every pixel-sample is finished exactly once after the right number of sweeps, the loop ends,
and the shaded waves hold one class unless leftovers were promoted."""
import numpy as np
import pytest

NT, K = 256, 64


def scan_excl(v):
    return np.concatenate([[0], np.cumsum(v)[:-1]])


def run_pool(P, minshade, q_total, max_bounces, nclass, p_miss, seed):
    rng = np.random.default_rng(seed)
    probs = rng.dirichlet(np.ones(nclass) * 0.7)
    rec_key = np.zeros(P, int)          # class key of the record (0: none)
    rec_wait = np.zeros(P, bool)
    rec_path = [None] * P               # (q, depth) of the record
    q_head = slot_head = 0
    my_slot = -np.ones(NT, int)
    have = np.zeros(NT, bool)
    q_done = np.full(NT, q_total == 0)
    path = [None] * NT                  # lane registers: [q, depth]
    sweeps = np.zeros(q_total, int)
    finished = np.zeros(q_total, int)
    rounds = mixed_waves = shaded_waves = 0
    cnt_ph = [np.zeros(K, int), np.zeros(K, int)]
    ph = 0
    if max_bounces < 1:  # the kernel stages a zero radiance for every pixel-sample and returns
        return np.ones(q_total, int), sweeps, 0, 0, 0
    while True:
        rounds += 1
        assert rounds < 100000, "the loop does not end"
        waves = list(range(4))
        # (1) slots: one atomic per wave, waves in a random order
        rng.shuffle(waves)
        for w in waves:
            lanes = [l for l in range(64 * w, 64 * w + 64) if not have[l] and my_slot[l] < 0 and not q_done[l]]
            base, slot_head = slot_head, slot_head + len(lanes)
            for i, l in enumerate(lanes):
                my_slot[l] = base + i if base + i < P else -1
        swept = np.zeros(NT, bool)
        key = np.zeros(NT, int)
        rng.shuffle(waves)
        for w in waves:  # the refill-and-sweep loop of each wave
            while True:
                lanes = [l for l in range(64 * w, 64 * w + 64) if not have[l] and my_slot[l] >= 0 and not q_done[l]]
                base, q_head = q_head, q_head + len(lanes)
                for i, l in enumerate(lanes):
                    q = base + i
                    if q >= q_total:
                        q_done[l] = True
                    else:
                        path[l] = [q, 1]
                        have[l] = True
                do = [l for l in range(64 * w, 64 * w + 64) if have[l] and not swept[l]]
                if not do:
                    break
                for l in do:
                    q, d = path[l]
                    sweeps[q] += 1
                    if rng.random() < p_miss:
                        finished[q] += 1
                        have[l] = False
                    else:
                        key[l] = 1 + rng.choice(nclass, p=probs)
                        swept[l] = True
        # (2) records, counts (swept paths, then the owners' visits of waiting records), in a random lane order
        cnt = cnt_ph[ph]
        assert not cnt.any()
        rank = np.zeros(NT, int)
        carried = [my_slot[l] for l in range(NT) if swept[l]]
        assert len(set(carried)) == len(carried), "two lanes carry one slot"
        for l in range(NT):
            if swept[l]:
                s = my_slot[l]
                assert not rec_wait[s]
                rec_key[s], rec_path[s] = key[l], list(path[l])
        w_key = np.zeros((NT, 2), int)
        w_rank = -np.ones((NT, 2), int)
        events = [(l, None) for l in range(NT) if swept[l]] + [(s % NT, s) for s in range(P) if rec_wait[s]]
        rng.shuffle(events)
        for l, s in events:
            if s is None:
                rank[l] = cnt[key[l]]
                cnt[key[l]] += 1
            else:
                v = s // NT
                w_key[l, v] = rec_key[s]
                w_rank[l, v] = cnt[rec_key[s]]
                cnt[rec_key[s]] += 1
        # (3) placement
        live = cnt.sum()
        if live == 0:
            break
        no_work = q_head >= q_total
        pool_full = slot_head >= P
        full = cnt & ~63
        f_start = scan_excl(full)
        f_shade = np.minimum(full, np.maximum(NT - f_start, 0))
        n_full = f_shade.sum()
        promote = n_full < minshade and (pool_full or no_work)
        left = cnt - f_shade if promote else np.zeros(K, int)
        l_start = n_full + scan_excl(left)
        l_shade = np.minimum(left, np.maximum(NT - l_start, 0))
        n_shade = n_full + l_shade.sum()

        def place(k, r):
            if r < f_shade[k]:
                return f_start[k] + r
            if r - f_shade[k] < l_shade[k]:
                return l_start[k] + r - f_shade[k]
            return -1
        perm = -np.ones(NT, int)
        for l in range(NT):
            if swept[l]:
                pos = place(key[l], rank[l])
                if pos >= 0:
                    assert 0 <= pos < n_shade and perm[pos] < 0
                    perm[pos] = my_slot[l]
                else:
                    rec_wait[my_slot[l]] = True
            for v in range(2):
                if w_rank[l, v] >= 0:
                    s = l + v * NT
                    pos = place(w_key[l, v], w_rank[l, v])
                    if pos >= 0:
                        assert 0 <= pos < n_shade and perm[pos] < 0
                        perm[pos] = s
                        rec_wait[s] = False
        assert (perm[:n_shade] >= 0).all() and (perm[n_shade:] < 0).all()
        cnt[:] = 0
        ph ^= 1
        for w in range(0, n_shade, 64):
            ks = {rec_key[s] for s in perm[w:min(w + 64, n_shade)]}
            shaded_waves += 1
            mixed_waves += len(ks) > 1
            assert len(ks) == 1 or promote
        # (4) gather + shade
        for l in range(NT):
            if l < n_shade:
                s = perm[l]
                my_slot[l] = s
                q, d = rec_path[s]
                path[l] = [q, d]
                have[l] = True
                if d >= max_bounces:
                    finished[q] += 1
                    have[l] = False
                else:
                    path[l][1] = d + 1
            else:
                my_slot[l] = -1
                have[l] = False
    return finished, sweeps, rounds, mixed_waves, shaded_waves


@pytest.mark.parametrize("P,minshade,q_total,bounces,nclass,p_miss", [
    (320, 1, 256 * 4, 8, 6, 0.0),     # C3-like: closed room, six classes
    (288, 1, 256 * 4, 8, 3, 0.02),    # C2-like
    (320, 1, 200 * 3, 5, 9, 0.3),     # ragged block (200 pixels), many misses, more classes than fit
    (256, 1, 256 * 2, 16, 2, 0.01),
    (512, 256, 256 * 5, 3, 40, 0.1),  # promotion whenever fewer than 256 lanes would shade
    (320, 1, 0, 8, 4, 0.0),           # an empty block
    (320, 1, 256 * 2, 0, 4, 0.0),     # no bounce
    (300, 64, 37 * 2, 8, 5, 0.0),     # fewer paths than lanes
])
def test_pool_schedule_model(P, minshade, q_total, bounces, nclass, p_miss):
    for seed in range(3):
        finished, sweeps, rounds, mixed, waves = run_pool(P, minshade, q_total, bounces, nclass, p_miss, seed)
        assert (finished == 1).all(), "every pixel-sample ends exactly once"
        assert (sweeps <= max(bounces, 0)).all() and (sweeps >= min(bounces, 1)).all()
        if p_miss == 0.0:
            assert (sweeps == bounces).all()
