"""The rBRIEF sample slots k_describe blurs into (csrc/orb_slots.inc, read by make_desc_lanes) are data generated
by tools/gen/brief_slots.py; this pins the file to its generator and checks the properties the kernel relies on
(every pattern point's slot holds that point; each distinct point sits in one slot; the padding repeats a point).
The kernel also checks the first property at compile time (desc_slots_ok)."""
import importlib.util, os, re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "orb-slam-_amd", "csrc", "orb_slots.inc")


def _arrays():
    s = open(INC).read()
    get = lambda name: [int(x) for x in re.search(r"%s\[\d+\] = \{([^}]*)\}" % name, s).group(1).split(",")]
    return get("kSlotPt"), get("kPtSlot")


def _gen():
    spec = importlib.util.spec_from_file_location("brief_slots", os.path.join(ROOT, "tools", "gen", "brief_slots.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_slots_hold_their_points():
    slot_pt, pt_slot = _arrays()
    pts = _gen().pattern()
    assert len(slot_pt) == 384 and len(pt_slot) == 512
    for i in range(512):
        assert pts[slot_pt[pt_slot[i]]] == pts[i]
    distinct = {pts[i] for i in range(512)}
    assert len(distinct) == 375
    # each distinct point is referenced through exactly one slot
    used = {}
    for i in range(512):
        used.setdefault(pts[i], set()).add(pt_slot[i])
    assert all(len(v) == 1 for v in used.values())


def test_slots_match_generator():
    g = _gen()
    pts, slot_pts, pt_slot, _ = g.build()
    assert (slot_pts, pt_slot) == _arrays()
