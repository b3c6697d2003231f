"""``fluid.contrib.memory_usage`` (reference python/paddle/fluid/contrib/memory_usage_calc.py:46):
an estimate of a Program's activation memory at ``batch_size`` — the sum over the tensors its
ops write (each once), a -1 dim counted as ``batch_size`` — returned as (lower, upper, unit) with
the reference's 5 % / 10 % margins. The estimate ignores the executor's eager deletion (the
planner in static/program.py plan_program_memory gives the real peak)."""
from __future__ import annotations

__all__ = ["memory_usage"]


def memory_usage(program, batch_size):
    from ...static.program import Program, _iter_vars
    if not isinstance(program, Program):
        raise TypeError("Calculating Memory Usage requires Program as its Parameter. But you passed in %s"
                        % (type(program)))
    if batch_size <= 0:
        raise ValueError("The batch size need to be positive.")
    total, seen = 0.0, {"@EMPTY@"}
    for op in program.global_block().ops:
        for v in _iter_vars(op.outputs):
            if v.name in seen:
                continue
            seen.add(v.name)
            count, neg = 1, 0
            for d in v.shape:
                if d < 0:
                    neg += 1
                    if neg > 1:
                        raise ValueError("Var %s has more than one negative dim." % (v.name))
                    count *= batch_size * (-d)
                else:
                    count *= d
            total += count * v._t.element_size()
    unit = "B"
    if total > 1024:
        total /= 1024
        unit = "KB"
        if total > 1024:
            total /= 1024
            unit = "MB"
    return total * 1.05, total * 1.1, unit
