import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo")); sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
import numpy as np
from oracle import oracle as orc
import test_gpu_edges as T
tm, m, rm, tr, tips = T._setup("protein", compact=True)
st = T._oracle_state(orc, tm, m, rm, tr, tips)
ev, el, iv = m.engine_eigen()
P, S = st["partials"], st["scale"]
for p, a, b in tr.postorder_traversal[:: max(1, len(tr.postorder_traversal) // 5)]:
    for u, v in ((int(a), int(p)), (int(p), int(b))):
        site = tm.compute_likelihood_at_edge(u, v)
        rp, rs = tm.root_partials, tm.root_scale
        cml = np.zeros(rs.shape)
        rref = orc.clv(orc.pmatrix(ev, el, iv, 0.0, rm.rates), orc.pmatrix(ev, el, iv, tr.brlens[u, v], rm.rates), P[u], P[v], S[u], S[v], cml)
        vs = np.abs(rref).max(axis=-1)
        r = (np.abs(rp - rref).max(axis=-1) / vs)
        i = np.unravel_index(np.argmax(r), r.shape)
        print(u, v, "worst", r.max(), i, "vs", vs[i], "scale", rs[i], cml[i], "gp max", np.abs(rp[i]).max())
        gu, gsu = tm.node_partials(u); gv, gsv = tm.node_partials(v)
        print("   child u err", (np.abs(gu - P[u]).max(axis=-1)/np.abs(P[u]).max(axis=-1)).max(), "v err", (np.abs(gv - P[v]).max(axis=-1)/np.abs(P[v]).max(axis=-1)).max())
        print("   at worst: u vec", P[u][i][:6], gu[i][:6]); print("   v", P[v][i][:6], gv[i][:6], S[u][i], S[v][i], gsu[i], gsv[i])
        break
    break
