"""Test helper: TCP port blocks for sessions across emulated hosts
(127.0.0.x), drawn below the ephemeral range (32768+, where gloo's and the
kernel's own connections live) and checked before use.

A block is only handed out once every address in it could be bound at that
moment (SO_REUSEADDR, as the session's listener sets it). With a process
group, rank 0 draws the block, every rank checks its own addresses and the
group agrees; a block any rank cannot bind is dropped and a new one drawn.
So a port some other process holds (the failure of r03's GPU run,
'bind/listen tcp port ...: Address already in use') costs a redraw, not the
test."""
import random
import socket

LOW, HIGH, STEP = 20000, 32000, 16


def bindable(addrs):
    """Every (ip, port) can be bound now."""
    for ip, port in addrs:
        s = socket.socket()
        try:
            s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            s.bind((ip, port))
        except OSError:
            return False
        finally:
            s.close()
    return True


def draw_block(addrs_of, first=None, tries=200, rng=None):
    """A base port b such that every address of addrs_of(b) is bindable;
    `first` is tried first (tests force a taken port there)."""
    rng = rng or random.Random()
    cands = ([first] if first is not None else []) + \
        [rng.randrange(LOW, HIGH, STEP) for _ in range(tries)]
    for b in cands:
        if bindable(addrs_of(b)):
            return b
    raise RuntimeError("no bindable port block in %d draws" % len(cands))


def agreed_block(my_addrs_of, first=None, tries=50, group=None):
    """Over the initialised torch.distributed group: rank 0 draws a base
    (`first` on the first round, unchecked, so a test can force a taken one),
    broadcasts it, every rank checks its own addresses my_addrs_of(base), and
    all agree; a block any rank cannot bind is redrawn. Returns (base,
    rounds it took)."""
    import torch.distributed as dist
    rng = random.Random()
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    for attempt in range(tries):
        box = [None]
        if rank == 0:
            box[0] = first if (attempt == 0 and first is not None) else rng.randrange(LOW, HIGH, STEP)
        dist.broadcast_object_list(box, src=0, group=group)
        ok = bindable(my_addrs_of(box[0]))
        flags = [None] * world
        dist.all_gather_object(flags, ok, group=group)
        if all(flags):
            return box[0], attempt + 1
    raise RuntimeError("no port block every rank could bind in %d rounds" % tries)


def taken_port():
    """A listening socket on 127.0.0.1 in the drawn range, held by the
    caller (close it when done): (socket, port)."""
    rng = random.Random()
    for _ in range(200):
        p = rng.randrange(LOW, HIGH, STEP)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            s.listen(1)
            return s, p
        except OSError:
            s.close()
    raise RuntimeError("could not hold a port")
