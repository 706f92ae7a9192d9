"""Measured parity margins next to their bars.

``check(quantity, measured, bar, op)`` asserts ``measured op bar`` and records the pair under the
running test's id; ``tests/conftest.py`` writes every record of the session to the JSON file named
by ``MLI_MARGINS_OUT`` (the GPU-suite runs commit it under profiles/), so the margins the suite
actually measured sit beside the bars it asserts.
"""
import math
import os

RECORDS = []


def _test_id():
    return os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]


def check(quantity, measured, bar, op="<=", note=None):
    measured = float(measured)
    ok = {"<=": measured <= bar, "<": measured < bar, ">=": measured >= bar, ">": measured > bar}[op]
    rec = {"test": _test_id(), "quantity": quantity, "measured": measured if math.isfinite(measured) else str(measured),
           "op": op, "bar": bar, "ok": bool(ok)}
    if note:
        rec["note"] = note
    RECORDS.append(rec)
    assert ok, "%s: measured %r, bar %s %r" % (quantity, measured, op, bar)
    return measured
