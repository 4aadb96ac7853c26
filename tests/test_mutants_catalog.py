"""tools/mutants.py stays runnable: every mutant's original text is still in its source file (a refactor
that moves the code must update the catalogue), and every group has tests that exist."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

import mutants  # noqa: E402


def test_every_mutant_still_applies():
    for m in mutants.MUTANTS:
        src = open(os.path.join(REPO, m.path)).read()
        assert src.count(m.old) == 1, (m.group, m.path, m.old[:80])
        assert m.new != m.old
        assert not m.equivalent or m.why, m.old[:80]


def test_every_group_has_existing_tests():
    groups = {m.group for m in mutants.MUTANTS}
    assert groups == set(mutants.TESTS)
    for g, files in mutants.TESTS.items():
        assert files and all(os.path.exists(os.path.join(REPO, f)) for f in files), g
