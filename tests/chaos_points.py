"""Seeded kill points for the chaos tests (tests/test_chaos.py on CPU ranks,
tests/test_gpu_multirank.py::test_device_chaos on the shared GPU).

A scenario is 1-3 points drawn from a seed:
  * `mock=rank,version,seqno,trial`: the rank dies on entering op `seqno` of `version`
    (the same rank may die twice: its second point carries the next trial number);
  * `mock_die_serving=rank,version,seqno,trial,where`: a survivor dies while it serves the
    recovery of a rank killed at (version, seqno) -- the survivors are blocked in that op while
    the restarted rank loads its checkpoint and replays the results it missed.  `where`: 0 the
    first serving point, 1 after the routing decision, 2 once the first bytes of a host transfer
    left, 3 right before a device exchange.
Points that cannot fire (a trial number never reached) are harmless: every run must still end
with the closed-form model on every rank, or with the engine's explicit "Too many nodes went
down" when every holder of some data is gone.
"""
import random


def draw(seed, world, niter, nops, wheres=(0, 1, 2)):
    rng = random.Random(seed)
    points, kills, deaths = [], [], {}
    for _ in range(rng.randint(1, 3)):
        if kills and rng.random() < 0.5:
            a, v, s = rng.choice(kills)
            b = rng.choice([x for x in range(world) if x != a])
            t = deaths.get(b, 0)
            # survivors wait in the op of the death or, when it completed without the dead rank
            # (a tree broadcast), in the next one
            s2 = s + rng.randint(0, 1)
            points.append("mock_die_serving=%d,%d,%d,%d,%d" % (b, v, s2, t, rng.choice(wheres)))
            deaths[b] = t + 1
            continue
        if kills and rng.random() < 0.3:
            r = rng.choice(kills)[0]  # the same rank again, on its next attempt
        else:
            r = rng.randrange(world)
        v, s = rng.randrange(niter), rng.randrange(nops + 1)  # nops: the checkpoint itself
        t = deaths.get(r, 0)
        points.append("mock=%d,%d,%d,%d" % (r, v, s, t))
        deaths[r] = t + 1
        kills.append((r, v, s))
    return points
