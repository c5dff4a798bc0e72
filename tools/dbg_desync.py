"""Debug: two-peer desync case d2-lag14-i5: compare cells/reports of device and oracle each tick."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
from test_p2p_desync import *
d, lag, interval, sparse = 2, (1, 4), 5, False
S, T = 96, 12
inputs, na, nb = networks(S, T, d, lag)
oa, ob = oracle_peer(MASK_A, S, d, interval, sparse), oracle_peer(MASK_B, S, d, interval, sparse)
ga, gb = gpu_peer(MASK_A, S, d, interval, sparse), gpu_peer(MASK_B, S, d, interval, sparse)
dev = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
di = dev(inputs)
ua, ra, ub, rb = dev(na[0]), dev(na[1]), dev(nb[0]), dev(nb[1])
for t in range(T):
    ga.run_ticks(di[t:t + 1], ua[t:t + 1], ra)
    gb.run_ticks(di[t:t + 1], ub[t:t + 1], rb)
    for name, g, o, m, net in (("A", ga, oa, MASK_A, na), ("B", gb, ob, MASK_B, nb)):
        ost, olf, ona, ons = oracle_tick(o, m, inputs, net, t)
        tags, imgs, cs = g.read_cells()
        otags, oimgs, ocs = o.read_cells()
        bad = np.nonzero((cs != ocs).any(axis=2) | (tags != otags))
        if bad[0].size:
            print("tick", t, name, "cells differ at (slot, session):", list(zip(*bad))[:6])
            w, s = bad[0][0], bad[1][0]
            print("  tags", tags[w, s], otags[w, s], "cs", cs[w, s], ocs[w, s], "img equal", np.array_equal(imgs[w, s], oimgs[w, s]))
            print("  load frame", g.status()[1][s], olf[s], "nadv", g.status()[2][s], ona[s], "nsave", g.status()[3][s], ons[s])
    rep_a, rep_b = ga.take_checksum_reports(), gb.take_checksum_reports()
    (fa, ca), (fb, cb) = exchange_oracle(oa, ob)
    for name, rep, f, c in (("A", rep_a, fa, ca), ("B", rep_b, fb, cb)):
        gf, gc = dev_reports_as_oracle(rep)
        bad = np.nonzero((gc != c).any(-1) & (f >= 0))
        if bad[0].size:
            print("tick", t, name, "reports differ", list(zip(*bad))[:6], gf[bad][:3], f[bad][:3], gc[bad][:3], c[bad][:3])
    ga.receive_checksum_reports(1, rep_b)
    gb.receive_checksum_reports(0, rep_a)
print("done")
