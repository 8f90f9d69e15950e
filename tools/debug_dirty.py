"""Debug: which statuses of test_receive_soa_dirty_vs_oracle[3] differ."""
import sys
import numpy as np
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import patrol_amd as pa
from oracle import oracle as O
import _gen
from collections import Counter
SEC = 10**9
rng = np.random.default_rng(3)
K = 3000
g = pa.GPURepo(device=0, log2_slots=14)
o = O.Repo()
names0 = _gen.key_names(np.arange(K))
a0, t0, e0 = _gen.clean_states(rng, K)
created = _gen.T0 - rng.integers(0, SEC, K)
g.seed(names0, a0, t0, e0, created)
o.seed(names0, a0, t0, e0, created)
n = 40000
ids = _gen.zipf_ids(rng, n, K + 500)
names = _gen.key_names(ids)
a, t, e = _gen.dirty_states(rng, n)
now = _gen.T0 + 7 * SEC
out = g.receive_soa(names, a, t, e, now)
st, ra, rt, re = o.receive_soa(names, a, t, e, now)
bad = np.nonzero(out["status"] != st)[0]
print("bad", len(bad), "first", bad[:10], "gpu", out["status"][bad[:10]], "ref", st[bad[:10]])
first_dirty = int(np.argmax(st != 1)) if (st != 1).any() else n
print("first non-merged in ref", first_dirty)
cnt = Counter(ids[first_dirty:].tolist())
bk = Counter(ids[bad].tolist())
print("bad keys (key: bad count / suffix count):", [(k, v, cnt[k]) for k, v in bk.most_common(10)])
suf = np.arange(first_dirty, n)
for b in bad[:12]:
    k = ids[b]
    pos = np.nonzero(ids[first_dirty:] == k)[0] + first_dirty
    print("bad", b, "key", k, "rank", int(np.searchsorted(pos, b)), "of", len(pos), "gpu", out["status"][b], "ref", st[b],
          "neighbours gpu", out["status"][pos[-3:]], "ref", st[pos[-3:]])
rep = (st & 0x7F) == 2
ra_g = out["reply"]["a"]
badr = np.nonzero(rep & (ra_g != ra))[0]
print("bad replies", len(badr), "of", int(rep.sum()))
for b in badr[:12]:
    k = ids[b]
    pos = np.nonzero(ids[first_dirty:] == k)[0] + first_dirty
    print("badrep", b, "key", k, "rank", int(np.searchsorted(pos, b)), "of", len(pos), "gpu a", hex(int(ra_g[b])), "ref", hex(int(ra[b])),
          "gpu t", hex(int(out["reply"]["t"][b])), "ref t", hex(int(rt[b])), "e", int(out["reply"]["e"][b]), int(re[b]))
