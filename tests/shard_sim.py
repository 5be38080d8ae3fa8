"""CPU restatement of the sharded merge step -- TEST ONLY.

Mirrors, per shard, what the kernels do (llmtokenizer_amd/csrc/kernels.hip):
k_scan (candidate validation, greedy a==b run parity, neighbour deltas, the
shard-edge step), k_apply role A (span rewrite, retiring a first token owned
by the left shard), k_edges (edge record), and the replicated count update of
role B -- with the halo computed by the library's own shard_halo (the same
__host__ __device__ function the GPU runs in k_select).  The exchange is a
callback: in-process sums, or torch.distributed (gloo) across processes.
Checked against the oracle's RULE mode on the whole corpus.
"""
from collections import Counter

from llmtokenizer_amd import api

HOLE = 0xFFFFFFFF
MARK = 0xFFFFFFFF
EW = 16


def murmur_pair(a, b):
    def rotl(x, r):
        return ((x << r) | (x >> (32 - r))) & 0xFFFFFFFF
    c1, c2, h = 0xcc9e2d51, 0x1b873593, 0x9747b28c
    for k in (a, b):
        k = (k * c1) & 0xFFFFFFFF
        k = (rotl(k, 15) * c2) & 0xFFFFFFFF
        h ^= k
        h = (rotl(h, 13) * 5 + 0xe6546b64) & 0xFFFFFFFF
    h ^= 8
    h ^= h >> 16
    h = (h * 0x85ebca6b) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xc2b2ae35) & 0xFFFFFFFF
    h ^= h >> 16
    return h


def summary_B(D):
    B = 65536
    while True:
        t = 0.3 * B
        if D >= 1 and (D - 1) >= t:
            B *= 2
            continue
        return 2 * B if D >= t else B


def select(counts):
    """RULE-mode argmax: max count, then smallest bucket under B, then smallest key"""
    live = [(k, c) for k, c in counts.items() if c > 0]
    if not live:
        return None
    B = summary_B(len(live))
    best = None
    for (u, v), c in live:
        key = (c, -(murmur_pair(u, v) & (B - 1)), -((u << 32) | v))
        if best is None or key > best[0]:
            best = (key, u, v)
    if best[0][0] <= 1:
        return None
    return best[1], best[2]


class Shard:
    def __init__(self, data: bytes):
        self.n = len(data)
        self.tok = list(data)
        self.dist = [0] * self.n
        self.F1 = 0
        self.L1 = self.n - 1
        self.halo = None

    # -- lookups (k_scan's id_at / v_left / v_right)
    def id_at(self, p):
        h = self.halo
        if p < 0:
            return h["HL"][-1 - p] if p >= -3 else HOLE
        if p >= self.n:
            return h["HR"][p - self.n] if p - self.n < 3 else HOLE
        return self.tok[p]

    def v_left(self, p):
        if p <= 0:
            return p - 1
        e = p - 1
        if self.tok[e] != HOLE:
            return e
        d = self.dist[e]
        return -1 if d > e else e - d

    def v_right(self, p, ln):
        if p >= self.n:
            return p + 1
        q = p + ln
        return self.n if q >= self.n else q

    def record(self, tlen):
        """k_edges"""
        r = [0] * EW
        for m in range(3):
            r[1 + m] = r[4 + m] = HOLE
        if self.F1 < self.n:
            c, p = 0, self.F1
            while p <= self.L1 and c < 7:
                x = self.tok[p]
                if c < 3:
                    r[1 + c] = x
                p += tlen[x]
                c += 1
            r[0] = c
            p = self.L1
            for m in range(3):
                if p < 0:
                    break
                r[4 + m] = self.tok[p]
                p = self.v_left(p)
            last, trail, p = r[4], 0, self.L1
            while p >= 0 and self.tok[p] == last:
                trail += 1
                p = self.v_left(p)
            r[7] = trail
            r[8] = 1 if p < 0 else 0
        r[9] = self.n & 0xFFFFFFFF
        r[10] = self.n >> 32
        return r

    def scan(self, a, b, z, tlen):
        """k_scan: occurrence list, the four delta Counters, xleft"""
        n, tok, h = self.n, self.tok, self.halo
        la, lb = tlen[a], tlen[b]
        occ = []
        DL, DR, IL, IR = Counter(), Counter(), Counter(), Counter()
        for i in range(n):
            if tok[i] != a:
                continue
            j = i + la
            if not (j < n and tok[j] == b):
                continue
            if a != b:
                occ.append(i)
                ps = self.v_left(i)
                p = self.id_at(ps)
                if p != HOLE:
                    cov = p == b and self.id_at(self.v_left(ps)) == a
                    if not cov:
                        DL[p] += 1
                        IL[p] += 1
                k = self.v_right(j, lb)
                q = self.id_at(k)
                if q != HOLE:
                    DR[q] += 1
                    nocc = q == a and self.id_at(self.v_right(k, la)) == b
                    IR[z if nocc else q] += 1
            else:
                ps = self.v_left(i)
                p = self.id_at(ps)
                start, left, pos = True, p != HOLE, i
                if p == a:
                    start = ps < 0
                    left = False
                    if h["hlrun"] & 1:
                        pos = j
                m = 0
                while start:
                    jj = pos + la
                    if jj >= n or tok[jj] != a:
                        break
                    k = self.v_right(jj, la)
                    occ.append(pos)
                    q = self.id_at(k)
                    knext = q == a
                    if m == 0 and left:
                        DL[p] += 1
                        IL[p] += 1
                    if q != HOLE:
                        DR[q] += 1
                        nocc = knext and self.id_at(self.v_right(k, la)) == a
                        IR[z if nocc else q] += 1
                    if not knext or k >= n:
                        break
                    pos = k
                    m += 1
        xleft = None
        if self.F1 < n:
            F1 = self.F1
            if h["HL"][0] == a and tok[F1] == b and (a != b or (h["hlrun"] & 1)):
                xleft = F1
            i = self.L1
            if tok[i] == a and h["HR"][0] == b and (a != b or not (h["myidx"] & 1)):
                occ.append(i)
                ps = self.v_left(i)
                p = self.id_at(ps)
                cov = p == HOLE
                if not cov:
                    cov = (p == b and self.id_at(self.v_left(ps)) == a) if a != b else p == a
                if not cov:
                    DL[p] += 1
                    IL[p] += 1
                q = h["HR"][1]
                if q != HOLE:
                    DR[q] += 1
                    IR[z if (q == a and h["HR"][2] == b) else q] += 1
        return occ, (DL, DR, IL, IR), xleft

    def apply(self, occ, xleft, a, b, z, tlen):
        """k_apply role A"""
        n, la, lb = self.n, tlen[a], tlen[b]
        L1new = None
        for i in occ:
            j, k = i + la, i + la + lb
            self.tok[i] = z
            if j < n:
                self.tok[j] = HOLE
                if k - 1 < n:
                    self.dist[k - 1] = k - 1 - i
                if j == self.L1:
                    L1new = i
        if xleft is not None:
            self.tok[xleft] = HOLE
            end = xleft + lb
            if end - 1 < n:
                self.dist[end - 1] = MARK
            self.F1 = end if end < n else n
        if L1new is not None:
            self.L1 = L1new

    def ids(self):
        return [x for x in self.tok if x != HOLE]


def train_sharded(parts, max_merges, sum_counters, gather_records, first_shard, nshards, forced=None):
    """Train on this process's shards `parts` (list of bytes, shard indices
    first_shard..).  sum_counters(list of 4 Counters + R) -> global; gather_records
    (list of local records) -> all records.  Returns (merges, [ids per local shard])."""
    shards = [Shard(p) for p in parts]
    tlen = {x: 1 for x in range(256)}
    # initial counts: local byte pairs + the pair across each right edge
    recs = gather_records([s.record(tlen) for s in shards])
    local = Counter()
    for q, s in enumerate(shards):
        for i in range(s.n - 1):
            local[(s.tok[i], s.tok[i + 1])] += 1
        me = first_shard + q
        for t in range(me + 1, nshards):
            if recs[t][0]:
                local[(s.tok[s.n - 1], recs[t][1])] += 1
                break
    counts = Counter(sum_counters([local])[0])
    merges = []
    z = 256
    while max_merges < 0 or len(merges) < max_merges:
        if forced is not None:  # encode: replay a given merge list
            if len(merges) == len(forced):
                break
            w = forced[len(merges)]
        else:
            w = select(counts)
        if w is None:
            break
        a, b = w
        if not (a < z and b < z):  # invalid record: no occurrence (tlen 1)
            merges.append((a, b))
            tlen[z] = 1
            recs = gather_records([s.record(tlen) for s in shards])
            z += 1
            continue
        merges.append((a, b))
        tlen[z] = tlen[a] + tlen[b]
        for q, s in enumerate(shards):
            s.halo = api.shard_halo(recs, first_shard + q, a)
        res = [s.scan(a, b, z, tlen) for s in shards]
        tot = Counter()
        vec = [Counter(), Counter(), Counter(), Counter()]
        for occ, dv, _ in res:
            tot["R"] += len(occ)
            for v in range(4):
                vec[v].update(dv[v])
        g = sum_counters(vec + [tot])
        DL, DR, IL, IR, T = g
        for x, c in DR.items():
            counts[(b, x)] -= c
        for x, c in DL.items():
            counts[(x, a)] -= c
        for x, c in IR.items():
            counts[(z, x)] += c
        for x, c in IL.items():
            counts[(x, z)] += c
        counts[(a, b)] -= T["R"]
        assert all(c >= 0 for c in counts.values()), "negative pair count"
        for s, (occ, _, xl) in zip(shards, res):
            s.apply(occ, xl, a, b, z, tlen)
        recs = gather_records([s.record(tlen) for s in shards])
        z += 1
    return merges, [s.ids() for s in shards]


def local_exchange():
    """exchange callbacks for a single process holding every shard"""
    def sum_counters(cs):
        return cs

    def gather(recs):
        return recs
    return sum_counters, gather
