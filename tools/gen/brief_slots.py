"""Generate orb-slam-_amd/csrc/orb_slots.inc: where k_describe blurs each distinct rBRIEF sample point.

The 512 points of the ORB pattern (orb_pattern.inc) hold 375 distinct ones.  k_describe blurs each once, in
384 slots: slot 64 q + l is blurred by lane l in round q (q < 6) and its u16 result lands at u16 index
64 q + l of a table in LDS, from which test m = 64 wd + lane reads its two samples.  Two LDS access patterns
depend on where each point sits (MI355X_MICROARCH.md, LDS: a wave64 access is serviced as two 32-lane groups,
one cycle per distinct address on the busiest bank):
  * the blur reads of a round: a half-round's 32 points are read at their rotated positions in the
    row-blurred patch, so they are taken as a compact cluster (32 consecutive points in Hilbert order of
    the unrotated pattern): a rotation keeps a cluster compact, and close points spread over few columns
    and share addresses, whatever the keypoint's angle;
  * the table reads of a test word: each 32-lane group reads 32 slots, on bank (slot >> 1) mod 32; within
    each half-round the lane order is free, and a local search picks it to minimise the busiest bank over
    the 16 table reads (8 instructions x 2 groups).
Output (data only): kSlotPt[384], the pattern point index blurred in each slot, and kPtSlot[512], the slot
holding each pattern point's value.  Run: python3 tools/gen/brief_slots.py (rewrites the .inc)."""
import math, os, random, re, sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "orb-slam-_amd", "csrc")


def pattern():
    s = open(os.path.join(SRC, "orb_pattern.inc")).read()
    v = [int(x) for x in re.findall(r"-?\d+", re.sub(r"/\*.*?\*/", "", s, flags=re.S))]
    return [(v[i], v[i + 1]) for i in range(0, len(v), 2)]


def hilbert(p, n=32):
    x, y = p[0] + 16, p[1] + 16
    d, s = 0, n // 2
    while s > 0:
        rx, ry = (1 if x & s else 0), (1 if y & s else 0)
        d += s * s * ((3 * rx) ^ ry)
        if ry == 0:
            if rx == 1:
                x, y = s - 1 - x, s - 1 - y
            x, y = y, x
        s //= 2
    return d


def table_cost(slot_of_pt):
    """busiest-bank cycles summed over the 16 table-read groups"""
    c = 0
    for wd in range(4):
        for e in range(2):
            for g in range(2):
                banks = {}
                for l in range(32 * g, 32 * g + 32):
                    dw = slot_of_pt[2 * (64 * wd + l) + e] >> 1
                    banks.setdefault(dw % 32, set()).add(dw)
                c += max(len(v) for v in banks.values())
    return c


def blur_cost(slot_pts, pts, kTP=23, nang=48):
    """busiest-bank cycles of the four dword reads per round, averaged over angles"""
    tot = 0
    for ai in range(nang):
        ang = 2 * math.pi * ai / nang + 0.1
        a, b = math.cos(ang), math.sin(ang)
        for q in range(6):
            ad = []
            for l in range(64):
                px, py = pts[slot_pts[64 * q + l]]
                x, y = int(round(px * a - py * b)), int(round(px * b + py * a))
                ad.append((18 + x) * kTP + ((18 + y) >> 1))
            for k in range(4):
                for g in range(2):
                    banks = {}
                    for d in ad[32 * g:32 * g + 32]:
                        banks.setdefault((d + k) % 32, set()).add(d + k)
                    tot += max(len(v) for v in banks.values())
    return tot / nang


def build(seed=1, iters=60000):
    pts = pattern()
    first = {}
    for i, p in enumerate(pts):
        first.setdefault(p, i)
    reps = sorted(set(first.values()), key=lambda i: hilbert(pts[i]))   # distinct points, Hilbert order
    assert len(reps) <= 384
    reps += [reps[-1]] * (384 - len(reps))   # padding repeats the last point (same address: a broadcast)
    slot_pts = list(reps)

    def slot_map(sp):
        sl = {}
        for s, i in enumerate(sp):
            sl.setdefault(i, s)
        return [sl[first[p]] for p in pts]

    rng = random.Random(seed)
    cur = table_cost(slot_map(slot_pts))
    for _ in range(iters):
        h = rng.randrange(12)   # half-round: slots 32 h .. 32 h + 31
        i, j = 32 * h + rng.randrange(32), 32 * h + rng.randrange(32)
        if slot_pts[i] == slot_pts[j]:
            continue
        slot_pts[i], slot_pts[j] = slot_pts[j], slot_pts[i]
        c = table_cost(slot_map(slot_pts))
        if c <= cur:
            cur = c
        else:
            slot_pts[i], slot_pts[j] = slot_pts[j], slot_pts[i]
    return pts, slot_pts, slot_map(slot_pts), cur


def main():
    pts, slot_pts, pt_slot, tc = build()
    # the same points in first-use order, for the log
    fu = []
    for i, p in enumerate(pts):
        if all(pts[j] != p for j in fu):
            fu.append(i)
    fu += [fu[0]] * (384 - len(fu))
    print("table-read cycles: %d (first-use order %d, ideal 16)" % (tc, table_cost(
        [[s for s, i in enumerate(fu) if pts[i] == p][0] for p in pts])))
    print("blur-read cycles per keypoint: %.1f (first-use order %.1f, ideal 48)" % (
        blur_cost(slot_pts, pts), blur_cost(fu, pts)))
    with open(os.path.join(SRC, "orb_slots.inc"), "w") as f:
        f.write("// generated by tools/gen/brief_slots.py: rBRIEF sample slots (data, see the script's docstring)\n")
        f.write("constexpr int kSlotPt[384] = {%s};\n" % ",".join(map(str, slot_pts)))
        f.write("constexpr int kPtSlot[512] = {%s};\n" % ",".join(map(str, pt_slot)))


if __name__ == "__main__":
    main()
