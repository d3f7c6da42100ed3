"""CPU: the oracle reproduces the committed full-size fixtures
(tests/golden/fullsize.json) — the bench configurations at their bench sizes,
two launches each (about 25 s on 5 cores)."""
import json
import os

from golden import make_fullsize


def test_fullsize_fixtures_regenerate(oracle):
    want = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "fullsize.json")))
    got = make_fullsize.generate()
    for k in make_fullsize.CASES:
        assert got[k] == want[k], k
