"""numpy pairwise-sum order (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

The reference normalises priors with ``policy.sum()`` on float32 arrays
(self_play.py:160, :211) and on float64 arrays (self_play.py:170, :378).
numpy 2.2.6 reduces contiguous float arrays with ``pairwise_sum``
(numpy/_core/src/umath/loops_utils.h.src): below 8 elements a plain loop from
0; up to 128 elements eight interleaved accumulators combined as
((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) followed by the tail; above 128 a split at
n/2 rounded down to a multiple of 8.  Every addition rounds to the array
dtype.  The engine's device code follows the same schedule so that child
priors are bit-identical; ``tests/test_oracle_golden.py`` checks this
restatement against ``np.sum`` itself.
"""
import numpy as np


def pairwise_sum(a, dtype):
    dt = np.dtype(dtype).type
    n = len(a)
    if n < 8:
        res = dt(0.0)
        for i in range(n):
            res = dt(res + dt(a[i]))
        return res
    if n <= 128:
        r = [dt(a[j]) for j in range(8)]
        i = 8
        stop = n - (n % 8)
        while i < stop:
            for j in range(8):
                r[j] = dt(r[j] + dt(a[i + j]))
            i += 8
        res = dt(dt(dt(r[0] + r[1]) + dt(r[2] + r[3])) +
                 dt(dt(r[4] + r[5]) + dt(r[6] + r[7])))
        while i < n:
            res = dt(res + dt(a[i]))
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return dt(pairwise_sum(a[:n2], dtype) + pairwise_sum(a[n2:], dtype))
