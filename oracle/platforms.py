"""ORACLE — test infrastructure only (tests/, bench.py's cpu_baseline leg).  Never imported by the product.

Cluster platforms and the LMM systems their flows build, restated in Python from the reference's own files
for the parity checks of configs C4 / C5 — independently of the product's generator
(simgrid_amd/csrc/lmm_platforms.hpp), so that a GPU-vs-oracle comparison on a generated platform also checks
the product's routing and flow construction:

* FatTreeZone.cpp:41-60 (is_in_sub_tree), 62-129 (get_local_route: d-mod-k up, label-matching down — the
  down loop keeps scanning the ports of the switch it has just reached), 161-202 / 236-359 (nodes, labels,
  links, ports), 443-485 (add_processing_node / add_link: SPLITDUPLEX cables, host and switch limiters,
  the host loopbacks);
* DragonflyZone.cpp:26-35 (rank -> coordinates), 126-236 (routers and their node / green / black / blue
  links, the blue link of group pair (i, j) on router j of group i), 238-336 (minimal routing, with the
  reference's flat router indices);
* sg_platf.cpp:130-139 (a SPLITDUPLEX link is an _UP and a _DOWN link), 214-251 (the cluster's private
  loopback / limiter links);
* network_cm02.cpp:36-64, 165-279 (CM02 / LV08 flows: bandwidth factor 0.97 and weight_S 20537 for LV08,
  the back route at weight 0.05 with crosstraffic, penalty latency + sum(weight_S / bw) and the TCP-gamma
  bound gamma / (2 lat) once the latency is paid, network_cm02.cpp:105-146);
* ptask_L07.cpp:143-208, 239-255, 389-417 (L07 flows: both CPUs at weight 0, every route link at the flow
  size through expand_add, penalty 1 and the bound gamma / (2 lat size) once the latency is paid).

Only links a route can use become constraints (the reference's per-host cluster links and the switches'
loopbacks carry no element).  Flows are drawn from SplitMix64(seed * 0x9E3779B97F4A7C15 + 7): source, then
destination (mod the host count), then for L07 the size from the top 53 bits — the parameters of the
synthetic workload, the same convention on both sides.

The system is handed to the C++ oracle as an ordered list of API calls (constraint_new / unshare, then per
flow variable_new and its expand / expand_add calls: `oracle_build_flows`), so the oracle's own
System::expand semantics (element merging, concurrency) apply exactly as when a simulation calls them.
"""
import numpy as np

FAT_TREE, DRAGONFLY = 0, 1
SHARED, SPLITDUPLEX, FATPIPE = 0, 1, 2
CM02, LV08, L07 = 0, 1, 2
_M64 = (1 << 64) - 1


class SplitMix64:
    def __init__(self, seed):
        self.s = seed & _M64

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & _M64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
        return z ^ (z >> 31)


def _ints(s, n, what):
    parts = s.split(",")
    if n is not None and len(parts) != n:
        raise ValueError(what)
    out = []
    for x in parts:
        try:
            v = int(x)
        except ValueError:
            raise ValueError(what + x) from None
        if v <= 0:
            raise ValueError(what + x)
        out.append(v)
    return out


class _Links:
    def __init__(self):
        self.bw, self.lat, self.fat = [], [], []

    def new(self, bw, lat, policy):
        """sg_platf.cpp:130-139: (up, down) ids; one link unless SPLITDUPLEX."""
        up = len(self.bw)
        self.bw.append(bw)
        self.lat.append(lat)
        self.fat.append(policy == FATPIPE)
        if policy != SPLITDUPLEX:
            return up, up
        self.bw.append(bw)
        self.lat.append(lat)
        self.fat.append(False)
        return up, up + 1


class FatTree(_Links):
    def __init__(self, p):
        super().__init__()
        msg = "Fat trees are defined by the levels number and 3 vectors"
        parts = p["topo_parameters"].split(";")
        if len(parts) != 4:
            raise ValueError(msg)
        self.L = _ints(parts[0], 1, msg)[0]
        self.down = _ints(parts[1], self.L, msg)
        self.up = _ints(parts[2], self.L, msg)
        self.ports = _ints(parts[3], self.L, msg)
        loop = p["loopback_bw"] > 0 or p["loopback_lat"] > 0
        lim = p["limiter_bw"] > 0
        if loop and lim:  # FatTreeZone.cpp:446-462 + network_cm02.cpp:99: one bandwidth per non-wifi link
            raise ValueError("Non WIFI links must use only 1 bandwidth.")
        self.loop, self.lim = loop, lim
        L, down, up, ports = self.L, self.down, self.up, self.ports
        # nodes per level (FatTreeZone.cpp:236-262)
        per = [int(np.prod(down))]
        for i in range(L):
            per.append(int(np.prod(up[:i + 1])) * int(np.prod(down[i + 1:])))
        self.per = per
        self.n_hosts = per[0]
        # nodes: level, position, label, parents / children cable ids per port, loopback, limiter
        self.level, self.pos, self.label, self.parents, self.children = [], [], [], [], []
        self.loopback, self.limiter = [], []
        for h in range(self.n_hosts):
            self._node(0, h, up[0] * ports[0], 0)
            self.limiter[-1] = self.new(p["limiter_bw"], 0.0, SHARED)[0] if lim else -1
            self.loopback[-1] = self.new(p["loopback_bw"], p["loopback_lat"], FATPIPE)[0] if loop else -1
        for i in range(L):
            for j in range(per[i + 1]):
                npar = up[i + 1] * ports[i + 1] if i != L - 1 else 0
                self._node(i + 1, j, npar, down[i] * ports[i])
                self.limiter[-1] = self.new(p["limiter_bw"], 0.0, SHARED)[0] if lim else -1
        # labels: per level a mixed-radix counter, digit j counts to down[j] below the level, up[j] above
        k = 0
        for i in range(L + 1):
            cur = [0] * L
            radix = [down[j] if j + 1 > i else up[j] for j in range(L)]
            for _ in range(per[i]):
                self.label[k] = list(cur)
                for d in range(L):
                    cur[d] += 1
                    if cur[d] < radix[d]:
                        break
                    cur[d] = 0
                k += 1
        # cables, child by child in (level, position) order, every port towards every related parent
        self.cab_up_node, self.cab_down_node, self.cab_up_link, self.cab_down_link = [], [], [], []
        start = np.concatenate([[0], np.cumsum(per)]).astype(int)
        k = 0
        for i in range(L):
            for _ in range(per[i]):
                lv = self.level[k]
                for q in range(per[lv + 1]):
                    pa = int(start[lv + 1]) + q
                    if not self._related(pa, k):
                        continue
                    for port in range(ports[lv]):
                        pport = self.label[k][lv] + port * down[lv]
                        cport = self.label[pa][lv] + port * up[lv]
                        u, dn = self.new(p["bw"], p["lat"], p["policy"])
                        cid = len(self.cab_up_node)
                        self.cab_up_node.append(pa)
                        self.cab_down_node.append(k)
                        self.cab_up_link.append(u)
                        self.cab_down_link.append(dn)
                        self.children[pa][pport] = cid
                        self.parents[k][cport] = cid
                k += 1

    def _node(self, level, pos, nparents, nchildren):
        self.level.append(level)
        self.pos.append(pos)
        self.label.append([0] * self.L)
        self.parents.append([-1] * nparents)
        self.children.append([-1] * nchildren)
        self.loopback.append(-1)
        self.limiter.append(-1)

    def _related(self, parent, child):  # FatTreeZone.cpp:204-234
        if self.level[parent] != self.level[child] + 1:
            return False
        for i in range(self.L):
            if self.label[parent][i] != self.label[child][i] and i + 1 != self.level[parent]:
                return False
        return True

    def _in_sub_tree(self, root, node):  # FatTreeZone.cpp:41-60
        if self.level[root] <= self.level[node]:
            return False
        for i in range(self.level[node]):
            if self.label[root][i] != self.label[node][i]:
                return False
        for i in range(self.level[root], self.L):
            if self.label[root][i] != self.label[node][i]:
                return False
        return True

    def route(self, src, dst, want_lat=True):
        """FatTreeZone.cpp:62-129: (links in route order, latency of the latency-carrying ones)."""
        out, lat = [], 0.0
        if src == dst and self.loop:
            lb = self.loopback[src]
            return [lb], self.lat[lb]
        cur = src
        while not self._in_sub_tree(cur, dst):  # up: d-mod-k on the destination's position
            x = self.pos[dst]
            for i in range(self.level[cur]):
                x //= self.up[i]
            x %= self.up[self.level[cur]]
            cb = self.parents[cur][x]
            if cb < 0:
                raise RuntimeError("fat tree: missing up port")
            out.append(self.cab_up_link[cb])
            lat += self.lat[self.cab_up_link[cb]]
            if self.lim:
                out.append(self.limiter[cur])
            cur = self.cab_up_node[cb]
        while cur != dst:  # down: the port scan goes on on the switch it has just reached
            before = cur
            i = 0
            while i < len(self.children[cur]):
                lv = self.level[cur]
                if i % self.down[lv - 1] == self.label[dst][lv - 1]:
                    cb = self.children[cur][i]
                    if cb < 0:
                        raise RuntimeError("fat tree: missing down port")
                    out.append(self.cab_down_link[cb])
                    lat += self.lat[self.cab_down_link[cb]]
                    cur = self.cab_down_node[cb]
                    if self.lim:
                        out.append(self.limiter[cur])
                i += 1
            if cur == before:
                raise RuntimeError("fat tree: no route down")
        return out, lat


class Dragonfly(_Links):
    def __init__(self, p):
        super().__init__()
        parts = p["topo_parameters"].split(";")
        if len(parts) != 4:
            raise ValueError("Dragonfly are defined by the number of groups, chassis per groups, blades per chassis,"
                             " nodes per blade")
        lv = "Dragonfly topologies are defined by 3 levels with 2 elements each, and one with one element"
        (self.G, self.blue_n), (self.C, self.black_n), (self.B, self.green_n) = (
            _ints(parts[k], 2, lv) for k in range(3))
        self.N = _ints(parts[3], 1, "Last parameter is not the amount of nodes per blade:")[0]
        self.lpl = 2 if p["policy"] == SPLITDUPLEX else 1
        G, C, B, N, lpl = self.G, self.C, self.B, self.N, self.lpl
        self.n_hosts = G * C * B * N
        self.loop = p["loopback_bw"] > 0 or p["loopback_lat"] > 0
        self.lim = p["limiter_bw"] > 0
        self.loopback = np.full(self.n_hosts, -1, dtype=np.int64)
        self.limiter = np.full(self.n_hosts, -1, dtype=np.int64)
        for h in range(self.n_hosts):  # sg_platf.cpp:214-251
            if self.loop:
                self.loopback[h] = self.new(p["loopback_bw"], p["loopback_lat"], FATPIPE)[0]
            if self.lim:
                self.limiter[h] = self.new(p["limiter_bw"], 0.0, SHARED)[0]
        R = G * C * B  # routers, index (group, chassis, blade) -> (g C + c) B + b (DragonflyZone.cpp:126-133)
        self.my_nodes = np.full((R, lpl * N), -1, dtype=np.int64)
        self.green = np.full((R, B), -1, dtype=np.int64)
        self.black = np.full((R, C), -1, dtype=np.int64)
        self.blue = np.full(R, -1, dtype=np.int64)
        for i in range(R):  # DragonflyZone.cpp:158-236
            for j in range(N):
                u, d = self.new(p["bw"], p["lat"], p["policy"])
                self.my_nodes[i, j * lpl] = u
                if lpl == 2:
                    self.my_nodes[i, j * lpl + 1] = d
        for i in range(G * C):
            for j in range(B):
                for k in range(j + 1, B):
                    u, d = self.new(p["bw"] * self.green_n, p["lat"], p["policy"])
                    self.green[i * B + j, k] = u
                    self.green[i * B + k, j] = d
        for i in range(G):
            for j in range(C):
                for k in range(j + 1, C):
                    for l in range(B):
                        u, d = self.new(p["bw"] * self.black_n, p["lat"], p["policy"])
                        self.black[i * B * C + j * B + l, k] = u
                        self.black[i * B * C + k * B + l, j] = d
        for i in range(G):
            for j in range(i + 1, G):
                ri, rj = i * B * C + j, j * B * C + i
                if ri >= R or rj >= R:
                    raise ValueError("dragonfly: more groups than routers per group")
                u, d = self.new(p["bw"] * self.blue_n, p["lat"], p["policy"])
                self.blue[ri] = u
                self.blue[rj] = d

    def coords(self, r):
        """DragonflyZone::rankId_to_coords (DragonflyZone.cpp:26-35) of host rank(s) r: (group, chassis, blade,
        node)."""
        C, B, N = self.C, self.B, self.N
        r = np.asarray(r, dtype=np.int64)
        return r // (C * B * N), r % (C * B * N) // (B * N), r % (B * N) // N, r % N

    def routes(self, src, dst):
        """DragonflyZone.cpp:238-336 for arrays of (src, dst): (link matrix padded with -1, in route order;
        latency of each route: the hops', not the limiters')."""
        G, C, B, N, lpl = self.G, self.C, self.B, self.N, self.lpl
        src = np.asarray(src, dtype=np.int64)
        dst = np.asarray(dst, dtype=np.int64)
        n = len(src)
        lat = np.array(self.lat)

        coords = self.coords  # DragonflyZone.cpp:26-35

        m0, m1, m2, m3 = coords(src)
        t0, t1, t2, t3 = coords(dst)
        cb = C * B
        me = m0 * cb + m1 * B + m2
        target = t0 * cb + t1 * B + t2
        cols, hops = [], []  # hops: whether the column's link carries latency (limiters do not)

        def put(link, mask, is_hop=True):
            if np.any(mask & (link < 0)):
                raise IndexError("dragonfly: no such link")
            cols.append(np.where(mask, link, -1))
            hops.append(is_hop)

        allm = np.ones(n, dtype=bool)
        put(self.my_nodes[me, m3 * lpl], allm)
        if self.lim:
            put(self.limiter[src], allm, False)
        far = target != me
        cur = me.copy()
        tg_group = t0  # router(target).group
        cur_group = m0
        inter = far & (tg_group != cur_group)
        # another group: to the blade that holds the blue link (green), to chassis 0 (black), blue link
        a = inter & (m2 != t0)
        put(self.green[cur, np.where(a, t0, 0)], a)
        cur = np.where(a, m0 * cb + m1 * B + t0, cur)
        chassis_cur = (cur % cb) // B
        b = inter & (chassis_cur != 0)
        put(self.black[cur, 0], b)
        cur = np.where(b, m0 * cb + t0, cur)
        put(self.blue[cur], inter)
        cur = np.where(inter, t0 * cb + m0, cur)
        # in the target group: blade (green), then chassis (black)
        c = far & (t2 != cur % B)
        put(self.green[cur, np.where(c, t2, 0)], c)
        cur = np.where(c, t0 * cb + t2, cur)
        d = far & (t1 != (cur % cb) // B)
        put(self.black[cur, np.where(d, t1, 0)], d)
        if self.lim:
            put(self.limiter[dst], allm, False)
        put(self.my_nodes[target, t3 * lpl + lpl - 1], allm)
        M = np.stack(cols, axis=1)
        L = np.zeros(n)
        for k, h in enumerate(hops):
            if h:
                L = L + np.where(M[:, k] >= 0, lat[np.maximum(M[:, k], 0)], 0.0)
        if self.loop:  # src == dst: the loopback alone
            same = src == dst
            if np.any(same):
                M[same] = -1
                M[same, 0] = self.loopback[src[same]]
                L[same] = lat[self.loopback[src[same]]]
        return M, L

    def route(self, src, dst, want_lat=True):
        M, L = self.routes([src], [dst])
        return [int(x) for x in M[0] if x >= 0], float(L[0])


def make_platform(p):
    if p["topology"] == FAT_TREE:
        return FatTree(p)
    if p["topology"] == DRAGONFLY:
        return Dragonfly(p)
    raise ValueError(f"unknown cluster topology {p['topology']}")


def platform_size(p):
    plat = make_platform(p)
    return len(plat.bw), plat.n_hosts


def _splitmix_stream(seed, n):
    """The first n outputs of SplitMix64(seed), vectorised: the state after k calls is seed + k * gamma."""
    g = np.uint64(0x9E3779B97F4A7C15)
    with np.errstate(over="ignore"):
        z = np.uint64(seed & _M64) + np.arange(1, n + 1, dtype=np.uint64) * g
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def flow_ops(p):
    """The API calls that build platform p's flows: constraints (bound, FATPIPE flag), and per flow the
    variable (penalty, bound, number of constraints) and its elements (constraint, weight, expand_add flag) in
    call order.  Returns a dict of numpy arrays (elements as a CSR over the flows)."""
    if p["model"] not in (CM02, LV08, L07):
        raise ValueError(f"unknown flow model {p['model']}")
    plat = make_platform(p)
    if plat.n_hosts <= 0:
        raise ValueError("platform without hosts")
    l07, lv08 = p["model"] == L07, p["model"] == LV08
    bw = np.array(plat.bw)
    factor = 1.0 if l07 else (0.97 if lv08 else 1.0)
    weight_s = 20537.0 if lv08 else 0.0
    cbound = [factor * b for b in plat.bw]
    cfat = list(plat.fat)
    cpu0 = len(cbound)
    if l07:
        cbound += [p["speed"]] * plat.n_hosts
        cfat += [False] * plat.n_hosts
    nf = int(p["n_flows"])
    per = 3 if l07 else 2  # RNG calls per flow: source, destination (, size)
    z = _splitmix_stream(p["seed"] * 0x9E3779B97F4A7C15 + 7, per * nf).reshape(nf, per) if nf else \
        np.zeros((0, per), dtype=np.uint64)
    src = (z[:, 0] % np.uint64(plat.n_hosts)).astype(np.int64)
    dst = (z[:, 1] % np.uint64(plat.n_hosts)).astype(np.int64)
    size = None
    if l07:
        size = p["size_min"] + (p["size_max"] - p["size_min"]) * (z[:, 2] >> np.uint64(11)).astype(np.float64) \
            * 2.0 ** -53
    back = not l07 and p["crosstraffic"]
    if isinstance(plat, Dragonfly):
        M, lat = plat.routes(src, dst)
        MB = plat.routes(dst, src)[0] if back else np.zeros((nf, 0), dtype=np.int64)
    else:  # fat tree: route by route (the down scan is not a closed form)
        rts, bks, lat = [], [], np.empty(nf)
        for f in range(nf):
            rt, lat[f] = plat.route(int(src[f]), int(dst[f]))
            rts.append(rt)
            if back:
                bks.append(plat.route(int(dst[f]), int(src[f]))[0])

        def pad(rows):
            w = max((len(r) for r in rows), default=0)
            out = np.full((nf, w), -1, dtype=np.int64)
            for f, r in enumerate(rows):
                out[f, :len(r)] = r
            return out
        M = pad(rts)
        MB = pad(bks) if back else np.zeros((nf, 0), dtype=np.int64)
    valid = M >= 0
    nr = valid.sum(axis=1)
    pos = lat > 0
    safe = np.where(pos, lat, 1.0)
    if l07:
        # penalty 1 once the latency is paid, and the bound updateBound sets then (ptask_L07.cpp:389-417)
        vpen = np.ones(nf)
        vbound = np.where(pos, p["tcp_gamma"] / (2.0 * safe * size), -1.0)
        srt = np.sort(np.where(valid, M, -1), axis=1)
        distinct = (srt >= 0) & np.concatenate([np.ones((nf, 1), dtype=bool), srt[:, 1:] != srt[:, :-1]], axis=1)
        vn = (2 + distinct.sum(axis=1)).astype(np.int32)
        C = np.concatenate([(cpu0 + src)[:, None], (cpu0 + dst)[:, None], M], axis=1)
        W = np.concatenate([np.zeros((nf, 2)), np.repeat(size[:, None], M.shape[1], axis=1)], axis=1)
        A = np.concatenate([np.zeros((nf, 2), dtype=np.uint8), np.ones(M.shape, dtype=np.uint8)], axis=1)
        mask = np.concatenate([np.ones((nf, 2), dtype=bool), valid], axis=1)
    else:
        pen = lat.copy()  # penalty = latency + sum(weight_S / bw) in route order, once the latency is paid
        for k in range(M.shape[1]):
            pen = pen + np.where(valid[:, k], weight_s / bw[np.maximum(M[:, k], 0)], 0.0)
        vpen = np.where(pos, pen, 1.0)
        vbound = np.where(pos, p["tcp_gamma"] / (2.0 * safe), -1.0)
        vb = MB >= 0
        vn = (nr + vb.sum(axis=1)).astype(np.int32)
        C = np.concatenate([M, MB], axis=1)
        W = np.concatenate([np.ones(M.shape), np.full(MB.shape, 0.05)], axis=1)
        A = np.zeros(C.shape, dtype=np.uint8)
        mask = np.concatenate([valid, vb], axis=1)
    eptr = np.concatenate([[0], np.cumsum(mask.sum(axis=1))]).astype(np.int64)
    return dict(cbound=np.array(cbound, dtype=np.float64), cfat=np.array(cfat, dtype=np.uint8),
                vpen=np.ascontiguousarray(vpen, dtype=np.float64), vbound=np.ascontiguousarray(vbound),
                vn=vn, eptr=eptr, ecnst=C[mask].astype(np.int32), ew=W[mask].astype(np.float64),
                eadd=A[mask].astype(np.uint8))


# ---- one link / one communication over explicit links (the pingpong replay, tests/pingpong_scenario.py) ----
def net_factors(model):
    """(latency factor, bandwidth factor, weight_S) of network_cm02.cpp:36-64: LV08 13.01 / 0.97 / 20537,
    CM02 1 / 1 / 0."""
    if model == LV08:
        return 13.01, 0.97, 20537.0
    if model == CM02:
        return 1.0, 1.0, 0.0
    raise ValueError(f"not a CM02-family network model: {model}")


def link_new(sys, model, bw, fatpipe=False):
    """NetworkCm02Link's constraint (network_cm02.cpp:282-295) on an oracle System: bandwidth factor * bw."""
    c = sys.constraint_new(None, net_factors(model)[1] * bw)
    if fatpipe:
        c.unshare()
    return c


def wifi_link_new(sys, model):
    """NetworkWifiLink's constraint (network_cm02.cpp:383-392): a NetworkCm02Link of bandwidth 1 / bandwidth
    factor, hence bound bandwidth factor * (1 / bandwidth factor); shared."""
    bf = net_factors(model)[1]
    return sys.constraint_new(None, bf * (1.0 / bf))


def communicate(sys, model, route, back=(), rate=-1.0, tcp_gamma=4194304.0, paid=False, crosstraffic=None):
    """NetworkCm02Model::communicate (network_cm02.cpp:165-274), its LMM part, on an oracle System:
    route = [(constraint, bw, lat)] in route order (route_to sums the latencies) — a WIFI access point as
    (constraint, bw, lat, (src_rate, dst_rate)), the stations' NetworkWifiLink::get_host_rate (-1: not
    associated), whose own bandwidth 1 / bandwidth factor and latency 0 replace bw / lat —, back = the back
    route's constraints (crosstraffic, weight 0.05).  Returns (variable, dict(latency, lat_current,
    sharing_penalty, bound)); the variable has penalty 0 while the latency is unpaid (1.0 without latency), or
    with `paid` the sharing penalty update_actions_state restores (network_cm02.cpp:105-146).  crosstraffic: the
    network/crosstraffic configuration (None: on iff `back` has links; the WIFI assertion of :242 tests the
    configuration, not the back route)."""
    if crosstraffic is None:
        crosstraffic = bool(len(back))
    lat_factor, bf, weight_s = net_factors(model)
    links = []
    for r in route:
        if len(r) > 3:  # WIFI: LinkImpl::get_bandwidth of the NetworkWifiLink, latency 0 (network_cm02.cpp:386)
            links.append((r[0], 1.0 / bf, 0.0, r[3]))
        else:
            links.append((r[0], r[1], r[2], None))
    lat = 0.0
    for _, _, l, _ in links:
        lat += l
    sharing_penalty = lat  # action->sharing_penalty_ = latency (network_cm02.cpp:188)
    if weight_s > 0:      # std::accumulate over the route (network_cm02.cpp:196-201)
        for _, bw, _, _ in links:
            sharing_penalty = sharing_penalty + weight_s / bw
    lat_current = lat
    latency = lat * lat_factor  # latency_ *= get_latency_factor(size) (network_cm02.cpp:208-209)
    if rate < 0:
        bound = tcp_gamma / (2.0 * lat_current) if lat_current > 0 else -1.0
    else:
        bound = min(rate, tcp_gamma / (2.0 * lat_current)) if lat_current > 0 else rate
    for _, _, _, rates in links:  # the assertions of network_cm02.cpp:242-255
        if rates is not None:
            if crosstraffic:
                raise ValueError("Cross-traffic is not yet supported when using WIFI")
            if rates[0] == -1 and rates[1] == -1:
                raise ValueError("Some Stations are not associated to any Access Point")
    pen = (sharing_penalty if paid else 0.0) if latency > 0 else 1.0
    v = sys.variable_new(None, pen, -1.0, len(links) + len(back))
    sys.update_variable_bound(v, bound)
    for c, _, _, rates in links:  # network_cm02.cpp:239-264
        if rates is None:
            w = 1.0
        elif rates[0] != -1:  # (src and dst on one access point: the source's rate, :249-251)
            w = 1.0 / rates[0]
        else:
            w = 1.0 / rates[1]
        sys.expand(c, v, w)
    for c in back:
        sys.expand(c, v, 0.05)
    return v, dict(latency=latency, lat_current=lat_current, sharing_penalty=sharing_penalty, bound=bound)
