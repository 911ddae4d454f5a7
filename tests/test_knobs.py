"""Every SS_* environment knob read anywhere in the sources is documented in
swiftsnails_amd/utils/knobs.py, and every documented knob is still read."""
import os
import re

from swiftsnails_amd.utils.knobs import KNOBS, table

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC_DIRS = ("swiftsnails_amd", "csrc")
SRC_FILES = ("bench.py", "__graft_entry__.py")
PAT = re.compile(r'"(SS_[A-Z0-9_]+)"')


def _read_knobs():
    found = {}
    paths = [os.path.join(ROOT, f) for f in SRC_FILES]
    for d in SRC_DIRS:
        for root, _, files in os.walk(os.path.join(ROOT, d)):
            paths += [os.path.join(root, f) for f in files
                      if f.endswith((".py", ".h", ".hip", ".cpp")) and f != "knobs.py"]
    for p in paths:
        with open(p, encoding="utf-8") as fh:
            for name in PAT.findall(fh.read()):
                found.setdefault(name, set()).add(os.path.relpath(p, ROOT))
    return found


def test_every_knob_is_documented_and_used():
    found = _read_knobs()
    undocumented = sorted(set(found) - set(KNOBS))
    stale = sorted(set(KNOBS) - set(found))
    assert not undocumented, f"add to utils/knobs.py: {undocumented} ({[found[k] for k in undocumented]})"
    assert not stale, f"no longer read anywhere: {stale}"


def test_knob_table_renders():
    t = table()
    assert t.count("\n") == len(KNOBS) + 1
    assert all(k.kind in ("ops", "tuning", "experiment", "debug", "build") for k in KNOBS.values())
