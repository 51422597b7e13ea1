"""Child-process helpers for the multi-process tests: one overall deadline
for all ranks, survivors killed and named (a dead rank left the
others waiting 300 s each, in turn, and the suite ran out of time)."""
import time


def join_all(ps, timeout):
    """Join every process against ONE deadline of `timeout` seconds, then kill
    whatever is still running. Returns the indices of the killed ones."""
    deadline = time.monotonic() + timeout
    for p in ps:
        p.join(max(0.0, deadline - time.monotonic()))
    hung = [i for i, p in enumerate(ps) if p.exitcode is None]
    for i in hung:
        ps[i].kill()
    for i in hung:
        ps[i].join(10)
    return hung


def hung_msg(hung, exitcodes):
    return "ranks %s still running at the deadline (killed); exit codes %s" % (hung, exitcodes)
