"""The arithmetic of one plan reduce item (ftar_internal.h ReduceItem), for the
numpy engine models in test_plan.py and test_dist_gloo.py: every fold step is
one reduce of the pinned oracle, so the models share the reference's
arithmetic exactly.

  round_each (the one-round ring): bf16 rounded after every add, one reduce per hop;
  shape (the one-round multi-stage tree): nested fold, one reduce per tree node;
  otherwise one k-way reduce (the staged schedules).
"""
import oracle_lib

BF16 = 9


def fold(item, srcs, dtype, op):
    if item.get("round_each") and dtype == BF16:
        out = srcs[0]
        for x in srcs[1:]:
            out = oracle_lib.reduce(dtype, op, [out, x])
        return out
    shape = item.get("shape", [])
    if len(shape) > 1:
        vals = list(srcs)
        for w in shape:
            vals = [oracle_lib.reduce(dtype, op, vals[i:i + w]) if w > 1 else vals[i]
                    for i in range(0, len(vals), w)]
        assert len(vals) == 1
        return vals[0]
    return oracle_lib.reduce(dtype, op, srcs)
