"""Tree-structured Parzen Estimator (TPE) search — own implementation.

``hyperopt`` is not available in this environment, so the TPE used by the
reference's Hyperopt drivers (reference
``cerebro_gpdb/run_ctq_hyperopt.py:76-91``,
``cerebro_gpdb/run_cerebro_standalone_helper.py:315-376``) is implemented here
with the same algorithmic shape as hyperopt 0.2's ``tpe.suggest``:

* the first ``n_startup`` suggestions are drawn from the prior,
* afterwards completed trials are split by loss into "good" (the best
  ``ceil(gamma * sqrt(n))``) and "bad", each dimension gets a Parzen density
  l(x) (good) and g(x) (bad) mixed with the prior, ``n_ei_candidates``
  samples are drawn from l(x) and the one maximising l(x)/g(x) is proposed.

Dimensions are independent (as in hyperopt).  Supported parameter kinds:
``choice``, ``uniform``, ``loguniform``, ``quniform``, ``randint``.
"""

import math

import numpy as np

STATUS_OK = "ok"
STATUS_RUNNING = "running"
STATUS_FAIL = "fail"


class Param(object):
    def __init__(self, name, kind, low=None, high=None, options=None, q=None):
        self.name, self.kind = name, kind
        self.low, self.high, self.options, self.q = low, high, options, q

    # internal representation: index for categorical, float otherwise
    def is_categorical(self):
        return self.kind in ("choice", "randint")

    def n_options(self):
        if self.kind == "choice":
            return len(self.options)
        return int(self.high - self.low)

    def to_value(self, internal):
        if self.kind == "choice":
            return self.options[int(internal)]
        if self.kind == "randint":
            return int(self.low + int(internal))
        if self.kind == "quniform":
            return float(np.round(internal / self.q) * self.q)
        return float(internal)

    def bounds(self):
        """Bounds in the space the Parzen estimator works in (log for loguniform)."""
        if self.kind == "loguniform":
            return math.log(self.low), math.log(self.high)
        return float(self.low), float(self.high)

    def to_work(self, internal):
        return math.log(internal) if self.kind == "loguniform" else float(internal)

    def from_work(self, w):
        return math.exp(w) if self.kind == "loguniform" else float(w)


def choice(name, options):
    return Param(name, "choice", options=list(options))


def uniform(name, low, high):
    return Param(name, "uniform", low, high)


def loguniform(name, low, high):
    """Log-uniform over [low, high] (note: takes the bounds, not their logs)."""
    return Param(name, "loguniform", low, high)


def quniform(name, low, high, q):
    return Param(name, "quniform", low, high, q=q)


def randint(name, low, high):
    """Integer in [low, high)."""
    return Param(name, "randint", low, high)


class Trials(object):
    """Trial documents: ``{'tid', 'vals': {name: internal}, 'status', 'loss'}``."""

    def __init__(self):
        self.trials = []

    def new_tid(self):
        return len(self.trials)

    def insert(self, vals, status=STATUS_RUNNING):
        doc = {"tid": self.new_tid(), "vals": dict(vals), "status": status, "loss": None}
        self.trials.append(doc)
        return doc

    def report(self, tid, loss, status=STATUS_OK):
        doc = self.trials[tid]
        doc["loss"] = float(loss) if loss is not None else None
        doc["status"] = status

    def completed(self):
        return [t for t in self.trials if t["status"] == STATUS_OK and t["loss"] is not None
                and np.isfinite(t["loss"])]

    def best(self):
        done = self.completed()
        return min(done, key=lambda t: t["loss"]) if done else None

    def __len__(self):
        return len(self.trials)


def _sample_prior(p, rng):
    if p.is_categorical():
        return int(rng.randint(p.n_options()))
    lo, hi = p.bounds()
    return p.from_work(rng.uniform(lo, hi))


def _parzen(mus, lo, hi, prior_weight):
    """Gaussian mixture (hyperopt adaptive_parzen_normal, simplified): prior
    component at the centre of the range with sigma = range, per-sample sigma
    = max gap to neighbours clipped to [range/min(100, n+1), range]."""
    prior_mu, prior_sigma = 0.5 * (lo + hi), (hi - lo)
    mus = np.asarray(mus, dtype=float)
    if len(mus) == 0:
        return np.array([prior_mu]), np.array([prior_sigma]), np.array([1.0])
    order = np.argsort(mus)
    srt = mus[order]
    all_mu = np.concatenate([[prior_mu], srt])
    all_mu_sorted_idx = np.argsort(all_mu)
    s = all_mu[all_mu_sorted_idx]
    left = np.diff(s, prepend=s[0])
    right = np.diff(s, append=s[-1])
    sig_sorted = np.maximum(left, right)
    sigma = np.empty_like(sig_sorted)
    sigma[all_mu_sorted_idx] = sig_sorted
    minsig = (hi - lo) / min(100.0, len(all_mu) + 1.0)
    sigma = np.clip(sigma, minsig, hi - lo)
    sigma[0] = prior_sigma
    w = np.ones(len(all_mu))
    w[0] = prior_weight
    return all_mu, sigma, w / w.sum()


def _gmm_logpdf(x, mus, sigmas, weights, lo, hi):
    x = np.atleast_1d(x)[:, None]
    # truncated normal mass inside [lo, hi]
    from math import erf, sqrt
    z_hi = np.array([0.5 * (1 + erf((hi - m) / (s * sqrt(2)))) for m, s in zip(mus, sigmas)])
    z_lo = np.array([0.5 * (1 + erf((lo - m) / (s * sqrt(2)))) for m, s in zip(mus, sigmas)])
    mass = np.maximum(z_hi - z_lo, 1e-12)
    dens = weights * np.exp(-0.5 * ((x - mus) / sigmas) ** 2) / (sigmas * math.sqrt(2 * math.pi)) / mass
    return np.log(np.maximum(dens.sum(axis=1), 1e-300))


def _gmm_sample(n, mus, sigmas, weights, lo, hi, rng):
    out = []
    while len(out) < n:
        k = rng.choice(len(mus), p=weights)
        v = rng.normal(mus[k], sigmas[k])
        if lo <= v <= hi:
            out.append(v)
    return np.array(out)


def tpe_suggest(space, trials, rng, n_startup=20, gamma=0.25, n_ei_candidates=24,
                prior_weight=1.0):
    """Propose one configuration (internal values) given completed trials."""
    done = trials.completed()
    if len(done) < n_startup:
        return {name: _sample_prior(p, rng) for name, p in space.items()}
    losses = np.array([t["loss"] for t in done])
    n_below = int(math.ceil(gamma * math.sqrt(len(done))))
    order = np.argsort(losses, kind="stable")
    below = [done[i] for i in order[:n_below]]
    above = [done[i] for i in order[n_below:]]
    proposal = {}
    for name, p in space.items():
        if p.is_categorical():
            K = p.n_options()
            cb = np.bincount([int(t["vals"][name]) for t in below], minlength=K).astype(float)
            ca = np.bincount([int(t["vals"][name]) for t in above], minlength=K).astype(float)
            lw = (cb + prior_weight) / (cb + prior_weight).sum()
            gw = (ca + prior_weight) / (ca + prior_weight).sum()
            cands = rng.choice(K, size=n_ei_candidates, p=lw)
            score = np.log(lw[cands]) - np.log(gw[cands])
            proposal[name] = int(cands[int(np.argmax(score))])
        else:
            lo, hi = p.bounds()
            bm, bs, bw = _parzen([p.to_work(t["vals"][name]) for t in below], lo, hi, prior_weight)
            am, as_, aw = _parzen([p.to_work(t["vals"][name]) for t in above], lo, hi, prior_weight)
            cands = _gmm_sample(n_ei_candidates, bm, bs, bw, lo, hi, rng)
            score = _gmm_logpdf(cands, bm, bs, bw, lo, hi) - _gmm_logpdf(cands, am, as_, aw, lo, hi)
            proposal[name] = p.from_work(float(cands[int(np.argmax(score))]))
    return proposal


def vals_to_params(space, vals):
    return {name: space[name].to_value(v) for name, v in vals.items()}


def fmin(fn, space, max_evals, rng=None, trials=None, **tpe_kw):
    """Sequential minimisation helper (hyperopt.fmin analogue, TPE only)."""
    rng = rng if rng is not None else np.random.RandomState(2018)
    trials = trials if trials is not None else Trials()
    while len(trials) < max_evals:
        vals = tpe_suggest(space, trials, rng, **tpe_kw)
        doc = trials.insert(vals)
        loss = fn(vals_to_params(space, vals))
        trials.report(doc["tid"], loss)
    best = trials.best()
    return vals_to_params(space, best["vals"]) if best else None, trials
