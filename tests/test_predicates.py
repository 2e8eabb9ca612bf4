"""The traversal's single-precision forms of the reference's double epsilon
compares (csrc/rt_predicates.h) equal the double forms on every input class:
edge sets (powers of two and neighbours in every binade, tiny, denormal,
infinite, NaN, equal operands) and 4e7 random pairs."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


import pytest


@pytest.mark.parametrize("fast", [False, True])
def test_fast_predicates_equal_double_forms(tmp_path, fast):
    """Built both ways: with -DRT_FAST_PREDICATES the unguarded fast forms
    (enter, lt_eps, gt_eps, add_eps) are checked too; the guarded float forms
    the traversal uses (split_safe / entry_safe + *_f) in both builds."""
    exe = str(tmp_path / "predicates_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", *(["-DRT_FAST_PREDICATES"] if fast else []),
                    "-o", exe, os.path.join(HERE, "predicates_check.cpp")], check=True)
    r = subprocess.run([exe, "20000000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout
