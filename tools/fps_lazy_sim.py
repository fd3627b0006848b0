"""Eager vs lazy bucket updates for exact FPS (numpy simulation, CPU).

eager: every step refreshes each bucket whose box lower bound to the new sample q is below its max.
lazy : a bucket hit by q (lb < its upper bound UB) is only *marked* (q appended to its pending list);
       it is refreshed — its points' dist brought up to date against every pending sample, one load
       of its points — only when its UB exceeds L_w, the largest exact max among the buckets of its
       wave that q did not touch (a lower bound of the new frame maximum, so a bucket left stale can
       never hold the argmax).  Pending lists are capped at CAP samples (overflow forces a refresh).
Reports bucket loads per step (traffic ~ loads x S x 16 B), sample evaluations per point loaded and
the pending-list lengths at refresh.  usage: fps_lazy_sim.py STEPS S WAVES CAP"""
import sys
import numpy as np

rng = np.random.default_rng(1)
N = 65536
M = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
S = int(sys.argv[2]) if len(sys.argv) > 2 else 16
WAVES = int(sys.argv[3]) if len(sys.argv) > 3 else 8
CAP = int(sys.argv[4]) if len(sys.argv) > 4 else 8
MODE = sys.argv[5] if len(sys.argv) > 5 else "wave"  # wave | global | cand
x = rng.uniform(-1, 1, (N, 3)).astype(np.float32)


def spread(v, bits):
    r = np.zeros_like(v)
    for b in range(bits):
        r |= ((v >> b) & 1) << (3 * b)
    return r


lo = x.min(0)
hi = x.max(0)
c = np.clip(((x - lo) * (32 / (hi - lo))).astype(np.int64), 0, 31)
order = np.argsort(spread(c[:, 0], 5) | (spread(c[:, 1], 5) << 1) | (spread(c[:, 2], 5) << 2), kind="stable")
xs = x[order]
nb = N // S
P = xs.reshape(nb, S, 3)
bmin = P.min(1)
bmax = P.max(1)
wave_of = np.arange(nb) % WAVES


def lbs(q):
    g = np.maximum(np.maximum(bmin - q, q - bmax), 0)
    return (g * g).sum(1)


def d2(pts, q):
    return ((pts - q) ** 2).sum(-1).astype(np.float32)


# eager reference
dist_e = np.full((nb, S), np.inf, np.float32)
# lazy state
dist_l = np.full((nb, S), np.inf, np.float32)
ub = np.full(nb, np.inf, np.float32)      # >= true bucket max
exact = np.ones(nb, bool)                 # ub == true max
pending = [[] for _ in range(nb)]
last_e = last_l = 0
loads_e = loads_l = 0
evals_l = 0
plen = []
wmax = []
emax = []
for it in range(1, M):
    qe = P.reshape(-1, 3)[last_e]
    a = lbs(qe) < dist_e.max(1)
    loads_e += int(a.sum())
    dist_e[a] = np.minimum(dist_e[a], d2(P[a], qe))
    last_e = int(np.argmax(dist_e.reshape(-1)))

    q = P.reshape(-1, 3)[last_l]
    hit = lbs(q) < ub
    for b in np.nonzero(hit)[0]:
        pending[b].append(q)
        exact[b] = False
    # per-wave lower bound of the new maximum: exact buckets q did not touch
    L = np.full(WAVES, -1.0, np.float32)
    for w in range(WAVES):
        m = (wave_of == w) & exact
        if m.any():
            L[w] = ub[m].max()
    if MODE == "global":
        Lb = np.full(WAVES, L.max())
    elif MODE == "cand":  # the previous step's wave candidates, each brought up to date against q
        Lg = max(min(cd, float(((cp - q) ** 2).sum())) for cd, cp in cands) if it > 1 else -1.0
        Lb = np.maximum(L, Lg)
    else:
        Lb = L
    need = (~exact) & ((ub >= Lb[wave_of]) | np.array([len(p) > CAP for p in pending]))
    per_wave = np.bincount(wave_of[need], minlength=WAVES)
    wmax.append(per_wave.max())
    act_w = np.bincount(wave_of[a], minlength=WAVES)
    emax.append(act_w.max())
    for b in np.nonzero(need)[0]:
        qs = np.array(pending[b], np.float32)
        plen.append(len(qs))
        evals_l += len(qs) * S
        dd = ((P[b][:, None, :] - qs[None, :, :]) ** 2).sum(-1).astype(np.float32).min(1)
        dist_l[b] = np.minimum(dist_l[b], dd)
        ub[b] = dist_l[b].max()
        exact[b] = True
        pending[b] = []
    loads_l += int(need.sum())
    # argmax over exact buckets only (stale ones have ub <= L <= max)
    flat = np.where(exact[:, None], dist_l, -1.0).reshape(-1)
    last_l = int(np.argmax(flat))
    cands = []
    for w in range(WAVES):
        fw = np.where((wave_of == w)[:, None] & exact[:, None], dist_l, -1.0).reshape(-1)
        j = int(np.argmax(fw))
        cands.append((float(fw[j]), P.reshape(-1, 3)[j].astype(np.float64)))
    assert last_l == last_e, (it, last_l, last_e)
print("max per wave per step: eager %.2f lazy %.2f" % (np.mean(emax), np.mean(wmax)))
print("S=%d waves=%d cap=%d steps=%d: eager loads/step %.1f (%.0f pts)  lazy loads/step %.1f (%.0f pts)  "
      "lazy evals/pt-loaded %.2f  pending mean %.2f max %d"
      % (S, WAVES, CAP, M, loads_e / (M - 1), loads_e * S / (M - 1), loads_l / (M - 1), loads_l * S / (M - 1),
         evals_l / max(1, loads_l * S), np.mean(plen), max(plen)))
