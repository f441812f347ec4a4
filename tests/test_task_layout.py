"""CPU model of traceTileTasks' sorted-path layout (sail_trace.hip): the per-key counts of a workgroup become key
starts in which every shading class begins a new 64-lane task, and each task finds its class by a search over the
classes' last keys. The model restates the kernel's per-lane formulas (prefix sums, running maximum, padded class
sizes) and checks, over random scenes and counts, that every path gets its own slot, every task holds one class,
and a task lane reads a slot only if a path was written there. (A first version took every key that is not its
class's last as a candidate of the search; on the GPU it read unwritten slots -- this model reproduces that.)"""
import random


def _scan(v):
    out, acc = [], 0
    for x in v:
        acc += x
        out.append(acc)
    return out


def _layout(seg_of_key, counts, k_max_tasks=12, last_candidate_only=True):
    first = [lane == 0 or seg_of_key[lane] != seg_of_key[lane - 1] for lane in range(64)]
    last = [lane == 63 or seg_of_key[lane + 1] != seg_of_key[lane] for lane in range(64)]
    incl = _scan(counts)
    excl = [a - b for a, b in zip(incl, counts)]
    n_alive = incl[63]
    base, m = [], 0
    for e, f in zip(excl, first):
        m = max(m, e if f else 0)
        base.append(m)
    total = [a - b for a, b in zip(incl, base)]
    R = [((t + 63) & ~63) if la else 0 for t, la in zip(total, last)]
    r_incl = _scan(R)
    padded = r_incl[63] <= k_max_tasks * 64
    n_tasks = r_incl[63] >> 6 if padded else (n_alive + 63) >> 6
    key_start = [(ri - r) + (e - b) if padded else e for ri, r, e, b in zip(r_incl, R, excl, base)]
    miss = -1 if last_candidate_only else 0x7FFFFFFF
    class_end = [ri if la else miss for ri, la in zip(r_incl, last)]
    class_info = [(t | (r << 16)) if la else 0 for t, r, la in zip(total, R, last)]
    perm = {}
    for k in range(64):
        for rank in range(counts[k]):
            d = key_start[k] + rank
            assert d not in perm
            perm[d] = k
    read = set()
    for tk in range(n_tasks):
        cand = [lane for lane in range(64) if class_end[lane] > tk * 64]
        L = cand[0]
        end, info = class_end[L], class_info[L]
        for lane in range(64):
            slot = tk * 64 + lane
            on = (slot - (end - (info >> 16)) < (info & 0xFFFF)) if padded else slot < n_alive
            if on:
                if slot not in perm:
                    return False
                read.add(slot)
        if padded:
            assert len({seg_of_key[perm[s]] for s in range(tk * 64, tk * 64 + 64) if s in perm}) <= 1
    assert read == set(perm)
    return True


def _random_case(rng):
    n = rng.randint(1, 63)
    segs, cur = [0], 0
    for k in range(1, n + 1):
        if k == 1 or rng.random() < 0.4:
            cur += 1
        segs.append(cur)
    segs += [cur + 1] * (63 - n)
    counts = [0] * 64
    for _ in range(rng.randint(0, 256)):
        counts[rng.randint(1, n)] += 1
    return segs, counts


def test_task_layout_covers_every_path_once():
    rng = random.Random(7)
    for _ in range(3000):
        segs, counts = _random_case(rng)
        assert _layout(segs, counts)
        generic = [(lane + 9) // 10 for lane in range(64)]  # (material, shape) keys: a class per material
        c2 = [0] * 64
        for _ in range(rng.randint(0, 256)):
            c2[rng.randint(1, 50)] += 1
        assert _layout(generic, c2)


def test_task_layout_first_version_read_unwritten_slots():
    rng = random.Random(7)
    assert any(not _layout(*_random_case(rng), last_candidate_only=False) for _ in range(200))
