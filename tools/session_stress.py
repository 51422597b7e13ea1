#!/usr/bin/env python3
"""Repeat the any-order async session test (tests/test_session.py
_run_any_order: every rank starts the same names in its own random order,
`steps` steps back to back) many times — host mode on the CPU, device mode on
the GPU box — to shake out rare interleavings of the concurrent async path.

    python tools/session_stress.py host 20
    python tools/session_stress.py device 6
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "tests")]


def main():
    mode, reps = sys.argv[1], int(sys.argv[2])
    import test_session as ts
    configs = [(2, None), (3, None), (4, "RING"), (4, "CLIQUE"), (3, "BINARY_TREE"),
               (4, "BINARY_TREE_STAR")]
    t0 = time.time()
    for rep in range(reps):
        for size, strategy in configs:
            ts._run_any_order(size, mode, strategy, steps=6)
        print("rep %d ok (%d configs x 6 steps, %.0f s)" % (rep, len(configs), time.time() - t0),
              flush=True)
    print("session stress ok: %s, %d reps" % (mode, reps))


if __name__ == "__main__":
    main()
