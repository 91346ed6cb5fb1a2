"""Boundary-velocity regressor of VBOC: the NN fit on the generated boundary states and its RMSE on
the held-out set.

Reference: my_nn.py:20-34 (NeuralNetDIR), VBOC/triplependulum_vboc.py:407-491 (first fit + RMSE),
:493-566 (refits as data arrives), the double VBOC/doublependulum_vboc.py:440-560 and the pendulum
VBOC/pendulum_vboc.py:35-41,228-292.

Model input = [ (q - mean) / std , qdot / |qdot| ], target = |qdot|  (:55-65); mean/std are the
scalar mean and (unbiased) std over ALL position entries, computed in float32 as the reference does
with torch.tensor(X[:, :nq].tolist()) (:50).  Training: Adam(lr 1e-3) on MSE, minibatch 4096 drawn
without replacement, EMA of the loss `val = 0.95 val + 0.05 loss` starting at max|qdot|; stop when
val <= 1e-3 or after it_max = 10 * int(n_0 * 100 / 4096) steps (:67-99), n_0 = size of the first
dataset (B and it_max are fixed once, :68-69).  Refits sample half of each minibatch from the old
rows and half from the new ones (:156-166).

MI355X design (the NN stays PyTorch-ROCm): the reference rebuilds each minibatch on
the host from Python lists (:164-165) and syncs on loss.item() every step.  Here the feature matrix
lives in HBM as float32, minibatch indices are drawn on the device (a uniform random k-subset = the
top-k of n uniform keys), and one training step - sampling, forward, backward, Adam, the EMA and the
stop test - is captured once in a HIP graph and replayed.  The stop test is evaluated on the device
and gates the update (a step taken after the stop condition is a no-op), so the host only polls the
`active` flag every `poll` steps while the iteration count and the final model are exactly those of
the reference's per-step loop.
"""
import math

import numpy as np
import torch
import torch.nn as nn


# ------------------------------------------------------------------------------------------------
# models (my_nn.py): same module structure, so state_dicts load in the reference's scripts
# ------------------------------------------------------------------------------------------------
class NeuralNetDIR(nn.Module):
    """my_nn.py:20-34: Linear-ReLU-Linear-ReLU-Linear-ReLU (non-negative output = |qdot|)."""

    def __init__(self, input_size, hidden_size, output_size):
        super().__init__()
        self.linear_relu_stack = nn.Sequential(
            nn.Linear(input_size, hidden_size), nn.ReLU(),
            nn.Linear(hidden_size, hidden_size), nn.ReLU(),
            nn.Linear(hidden_size, output_size), nn.ReLU())

    def forward(self, x):
        return self.linear_relu_stack(x)


class NeuralNetCLS(nn.Module):
    """my_nn.py:4-18 (the AL / HJR classifiers' architecture; loaded by the comparison scripts)."""

    def __init__(self, input_size, hidden_size, output_size):
        super().__init__()
        self.linear_relu_stack = nn.Sequential(
            nn.Linear(input_size, hidden_size), nn.ReLU(),
            nn.Linear(hidden_size, hidden_size), nn.ReLU(),
            nn.Linear(hidden_size, output_size))

    def forward(self, x):
        return self.linear_relu_stack(x)


# layer sizes per system: triple 6-500-1 (:38-41), double 4-300-1 (doublependulum_vboc.py:448-451),
# pendulum 2-100-1 (pendulum_vboc.py:35-37), minibatch 4096 / 4096 / 64
HIDDEN = {3: 500, 2: 300, 1: 100}
MINIBATCH = {3: 4096, 2: 4096, 1: 64}


# ------------------------------------------------------------------------------------------------
# data transforms
# ------------------------------------------------------------------------------------------------
def position_stats(X, nq):
    """(mean, std) of all position entries X[:, :nq], in float32 like
    torch.mean(torch.tensor(X[:, :nq].tolist())) (:50); returned as Python floats."""
    t = torch.from_numpy(np.ascontiguousarray(X[:, :nq], dtype=np.float64)).to(torch.float32)
    return torch.mean(t).item(), torch.std(t).item()


def dir_features(X, mean, std, nq):
    """[n, 2nq+1] float64: normalised positions, velocity direction (0 if qdot = 0), |qdot|
    (:55-65).  |qdot| is the sequential sum of squares; the reference's per-row numpy.linalg.norm
    can differ in the last bit of the float64 value, never after the cast to float32 the model sees."""
    X = np.asarray(X, dtype=np.float64)
    out = np.zeros((X.shape[0], 2 * nq + 1))
    out[:, :nq] = (X[:, :nq] - mean) / std
    V = X[:, nq:2 * nq]
    s = V[:, 0] * V[:, 0]
    for j in range(1, nq):
        s = s + V[:, j] * V[:, j]
    vn = np.sqrt(s)
    nz = vn != 0
    out[nz, nq:2 * nq] = V[nz] / vn[nz, None]
    out[:, 2 * nq] = vn
    return out


# ------------------------------------------------------------------------------------------------
# trainer
# ------------------------------------------------------------------------------------------------
class DirTrainer:
    """Adam/MSE fit of NeuralNetDIR with the reference's stop rule, device-resident.

    fit(F, n_new) trains on the feature matrix F ([n, 2nq+1], float) - the whole set for the first
    fit (:77-99), or old rows F[:n-n_new] and new rows F[n-n_new:] half-and-half for a refit
    (:156-184)."""

    def __init__(self, nq, device="cpu", hidden=None, minibatch=None, lr=1e-3, beta=0.95, stop_val=1e-3,
                 seed=0, graphs=None, poll=64):
        self.nq = nq
        self.nin = 2 * nq
        self.device = torch.device(device)
        torch.manual_seed(seed)
        self.hidden = hidden or HIDDEN[nq]
        self.model = NeuralNetDIR(self.nin, self.hidden, 1).to(self.device)
        self.k = minibatch or MINIBATCH[nq]
        self.lr, self.beta, self.stop_val = lr, beta, stop_val
        self.b1, self.b2, self.eps = 0.9, 0.999, 1e-8       # torch.optim.Adam defaults (:44)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self.params = [p for p in self.model.parameters()]
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.step_t = torch.zeros((), device=self.device)   # Adam step count (device-side)
        self.graphs = (self.device.type == "cuda") if graphs is None else graphs
        self.poll = poll
        self.it_max = None
        self.total_steps = 0
        self.seed, self.fits = seed, 0
        # Every buffer a captured step writes or reads across fits is allocated ONCE, here, outside any capture:
        # the gradients (backward accumulates into them after an in-graph zero_(), instead of allocating them in
        # the graph's private pool, where a new capture would find the previous graph's blocks), and the stop
        # rule's state (val, it, it_lim, active: refilled per fit, never re-allocated).  See fit() for the sampler.
        for p in self.params:
            p.grad = torch.zeros_like(p)
        self.val = torch.zeros((), device=self.device)
        self.it = torch.ones((), dtype=torch.int64, device=self.device)
        self.it_lim = torch.zeros((), dtype=torch.int64, device=self.device)
        self.active = torch.ones((), dtype=torch.bool, device=self.device)

    # -- one gated step, written with device tensors only (capturable) ---------------------------------
    # top-k slices are kept at most this long: a uniform k-subset of a long range is the top-k of the per-chunk
    # top-k candidates (exactly the same index set as one top-k over all keys).  A refit of the triple's VBOC loop
    # at configs[2]'s scale faulted the GPU (illegal address, profiles/r03f_vboc_loop_fault.log) in the first fit
    # whose halves exceeded 2^20 rows; the fits before it (halves of 0.5M rows) had run in the same process.
    TOPK_CHUNK = 1 << 18

    def _sample(self, lo, hi, k, gen=None):
        n = hi - lo
        keys = torch.rand(n, device=self.device, generator=gen or self.gen)
        if n <= self.TOPK_CHUNK:
            return torch.topk(keys, k, sorted=False).indices + lo
        c = self.TOPK_CHUNK
        m = (n + c - 1) // c
        pad = torch.full((m * c - n,), -1.0, device=self.device)        # keys are in [0, 1): pads never win
        part = torch.topk(torch.cat([keys, pad]).view(m, c), k, dim=1, sorted=False)
        cand = part.indices + (torch.arange(m, device=self.device) * c).unsqueeze(1)
        best = torch.topk(part.values.reshape(-1), k, sorted=False).indices
        return cand.reshape(-1).index_select(0, best) + lo

    def _step(self, F, X, y, n, n_new, gen=None):
        if n_new:
            idx = torch.cat([self._sample(0, n - n_new, self.k // 2, gen), self._sample(n - n_new, n, self.k // 2, gen)])
        else:
            idx = self._sample(0, n, self.k, gen)
        xb = X.index_select(0, idx)
        yb = y.index_select(0, idx)
        active = (self.val > self.stop_val) & (self.it < self.it_lim)
        a = active.to(torch.float32)
        for p in self.params:
            p.grad.zero_()
        loss = torch.mean((self.model(xb) - yb) ** 2)
        loss.backward()
        grads = [p.grad for p in self.params]
        with torch.no_grad():
            # Adam, torch.optim.Adam's arithmetic (single-tensor path), every update scaled by the gate
            self.step_t.add_(a)
            w1 = a * (1 - self.b1)
            w2 = a * (1 - self.b2)
            for m, v, g in zip(self.m, self.v, grads):
                m.lerp_(g, w1)
                v.mul_(1 - w2).addcmul_(g * w2, g)
            t = torch.clamp(self.step_t, min=1.0)
            bc1 = 1 - torch.pow(self.b1, t)
            bc2s = torch.sqrt(1 - torch.pow(self.b2, t))
            step = -(a * self.lr) / bc1
            for p, m, v in zip(self.params, self.m, self.v):
                p.addcdiv_(m * step, v.sqrt().div_(bc2s).add_(self.eps))
            # the reference's EMA and counter (:95-96), gated as well
            self.val.copy_(torch.where(active, self.beta * self.val + (1 - self.beta) * loss.detach(), self.val))
            self.it.add_(active.to(self.it.dtype))
            self.active.copy_(active)

    def fit(self, F, n_new=0, it_max=None):
        """Train until val <= stop_val or it_max steps.  Returns dict(iterations, val)."""
        F = torch.as_tensor(np.asarray(F), dtype=torch.float32).to(self.device) if not torch.is_tensor(F) \
            else F.to(self.device, torch.float32)
        n = F.shape[0]
        if self.it_max is None:
            B = int(n * 100 / self.k)   # :68, from the first dataset only
            self.it_max = B * 10
        it_max = it_max or self.it_max
        if n_new and (n_new < self.k // 2 or n - n_new < self.k // 2):
            raise ValueError("a refit needs at least minibatch/2 old and new rows")
        if not n_new and n < self.k:
            raise ValueError(f"need at least {self.k} rows (random.sample of a minibatch)")
        X = F[:, :self.nin].contiguous()
        y = F[:, self.nin:self.nin + 1].contiguous()
        self.val.copy_(torch.max(F[:, self.nin]))          # :73 val = max |qdot|
        self.it.fill_(1)
        self.it_lim.fill_(it_max)
        self.active.fill_(True)
        self.fits += 1
        steps = 0
        # Each fit draws from a generator of its own, seeded from the trainer's seed and the fit's index, in both
        # modes (so a captured fit equals the eager one).  A captured fit's graph is the only one that registers
        # it: re-registering one generator with a second graph after the first was destroyed is the pattern that
        # ran in the round-3 fault (profiles/r03f_vboc_loop_fault.log), and nothing of a
        # destroyed graph is referenced by the next one.
        gen = torch.Generator(device=self.device)
        gen.manual_seed(self.fit_seed(self.seed, self.fits))
        if self.graphs:
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):                      # warm-up outside capture (allocations)
                self._step(F, X, y, n, n_new, gen)
            torch.cuda.current_stream(self.device).wait_stream(s)
            steps += 1
            g = torch.cuda.CUDAGraph()
            g.register_generator_state(gen)                  # replays advance this fit's Philox offset
            with torch.cuda.graph(g):
                self._step(F, X, y, n, n_new, gen)
            while bool(self.active.item()):
                for _ in range(self.poll):
                    g.replay()
                steps += self.poll
            torch.cuda.synchronize(self.device)
            del g
        else:
            while bool(self.active.item()):
                self._step(F, X, y, n, n_new, gen)
                steps += 1
        self.total_steps += steps
        return dict(iterations=int(self.it.item()) - 1, val=float(self.val.item()), launched=steps)

    @staticmethod
    def fit_seed(seed, fit):
        """The seed of the minibatch generator of a trainer's fit number `fit` (1, 2, ...)."""
        return seed * 1_000_003 + fit

    @torch.no_grad()
    def predict(self, Xin, batch=1 << 15):
        """Model output for [n, 2nq] inputs in minibatches of 2^15 (VBOC/vboc.py:532-541)."""
        X = torch.as_tensor(np.asarray(Xin), dtype=torch.float32).to(self.device) if not torch.is_tensor(Xin) \
            else Xin.to(self.device, torch.float32)
        return torch.cat([self.model(X[i:i + batch]) for i in range(0, X.shape[0], batch)]) if X.shape[0] else \
            torch.zeros((0, 1), device=self.device)

    @torch.no_grad()
    def rmse(self, F):
        """sqrt(MSELoss(model(F[:, :2nq]), F[:, 2nq:])) (:117-120)."""
        F = torch.as_tensor(np.asarray(F), dtype=torch.float32).to(self.device) if not torch.is_tensor(F) \
            else F.to(self.device, torch.float32)
        out = self.predict(F[:, :self.nin])
        return math.sqrt(torch.mean((out - F[:, self.nin:self.nin + 1]) ** 2).item())


class HipTrainer(DirTrainer):
    """DirTrainer's fit on the device kernels of csrc/fit.hip (libvboc_fit.so, include/vboc_fit.h): sampling,
    forward, backward, Adam and the stop rule of VBOC/triplependulum_vboc.py:446-466 / :526-556 in four kernels
    per step, `poll` steps per HIP graph.  The torch module stays the source of truth between fits (its
    parameters are packed into the trainer before a fit and written back after it); Adam's moments and step count
    live in the trainer across fits, as the reference's one optimizer does.  Differences from DirTrainer: the
    minibatch draws (Philox, random.sample's redraw-on-repeat set method, instead of the top-k of uniform keys)
    and val, kept in float64 as the reference's Python float."""

    def __init__(self, nq, device="cuda", hidden=None, minibatch=None, lr=1e-3, beta=0.95, stop_val=1e-3, seed=0,
                 graphs=True, poll=64):
        import ctypes
        from . import fitlib
        super().__init__(nq, device, hidden=hidden, minibatch=minibatch, lr=lr, beta=beta, stop_val=stop_val,
                         seed=seed, graphs=False, poll=poll)
        if self.device.type != "cuda":
            raise ValueError("HipTrainer runs on a GPU (use DirTrainer on the CPU)")
        self._fl = fitlib
        self._lib = fitlib.load()
        h = ctypes.c_void_p()
        fitlib.check(self._lib.vboc_fit_create(self.nin, self.hidden, self.k, seed, ctypes.byref(h)))
        self._h = h
        self.use_graphs = graphs
        self.last = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.vboc_fit_destroy(h)
            self._h = None

    def _param_ptrs(self):
        st = self.model.linear_relu_stack
        ps = [st[0].weight, st[0].bias, st[2].weight, st[2].bias, st[4].weight, st[4].bias]
        for p in ps:
            if not p.is_contiguous() or p.dtype != torch.float32 or not p.is_cuda:
                raise ValueError("model parameters must be contiguous float32 tensors on the trainer's device")
        return [p.data_ptr() for p in ps]

    def fit(self, F, n_new=0, it_max=None):
        import ctypes
        fl = self._fl
        if torch.is_tensor(F):
            Ft = F.to(self.device, torch.float32).contiguous()
            val0 = float(Ft[:, self.nin].max())
        else:
            Fn = np.asarray(F)
            val0 = float(np.max(Fn[:, self.nin]))          # :446, over the float64 features
            Ft = torch.as_tensor(Fn, dtype=torch.float32).to(self.device).contiguous()
        n = Ft.shape[0]
        if self.it_max is None:
            self.it_max = int(n * 100 / self.k) * 10
        it_max = it_max or self.it_max
        if n_new and (n_new < self.k // 2 or n - n_new < self.k // 2):
            raise ValueError("a refit needs at least minibatch/2 old and new rows")
        if not n_new and n < self.k:
            raise ValueError(f"need at least {self.k} rows (random.sample of a minibatch)")
        stream = torch.cuda.current_stream(self.device).cuda_stream
        ptrs = self._param_ptrs()
        fl.check(self._lib.vboc_fit_set_params(self._h, *ptrs, stream))
        its, val, launched, ms = ctypes.c_longlong(), ctypes.c_double(), ctypes.c_longlong(), ctypes.c_double()
        run = fl.FitRun(F=Ft.data_ptr(), n=n, n_new=n_new, ld=Ft.shape[1], it_max=it_max, val0=val0,
                        stop_val=self.stop_val, beta=self.beta, lr=self.lr, poll=self.poll,
                        graphs=int(self.use_graphs), iterations=ctypes.addressof(its), val=ctypes.addressof(val),
                        launched=ctypes.addressof(launched), kernel_ms=ctypes.addressof(ms))
        fl.check(self._lib.vboc_fit_train(self._h, ctypes.byref(run), stream))
        fl.check(self._lib.vboc_fit_get_params(self._h, 0, *ptrs, stream))
        self.total_steps += launched.value
        self.last = dict(iterations=its.value, val=val.value, launched=launched.value, fit_ms=ms.value)
        return dict(iterations=its.value, val=val.value, launched=launched.value)

    def moments(self):
        """Adam's (exp_avg, exp_avg_sq) as lists of tensors in the model's parameter order (test hook)."""
        out = []
        stream = torch.cuda.current_stream(self.device).cuda_stream
        for which in (1, 2):
            ts = [torch.empty_like(p) for p in self.model.parameters()]
            self._fl.check(self._lib.vboc_fit_get_params(self._h, which, *[t.data_ptr() for t in ts], stream))
            out.append(ts)
        return out

    def sample(self, n, n_new=0, steps=1):
        """The sampler's next `steps` minibatches ([steps, k] int32 row indices; test hook)."""
        out = torch.empty((steps, self.k), dtype=torch.int32, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        self._fl.check(self._lib.vboc_fit_sample(self._h, n, n_new, steps, out.data_ptr(), stream))
        return out


def make_trainer(nq, device="cpu", native=False, **kw):
    """The fit of the VBOC loop: DirTrainer - PyTorch-ROCm, the reference's my_nn.py loop
    (VBOC/triplependulum_vboc.py:409-468) as north_star asks - by default.  native=True selects the native device
    trainer (HipTrainer, csrc/fit.hip) on a GPU for the shapes it implements (triple 6-500, double / Cartesian 4-300,
    pendulum 2-100, minibatch <= 4096; tests/test_fit_device.py pins it to torch Adam); other shapes and the CPU keep
    DirTrainer."""
    from . import fitlib
    dev = torch.device(device)
    hidden = kw.get("hidden") or HIDDEN.get(nq, 0)
    k = kw.get("minibatch") or MINIBATCH.get(nq, 0)
    if native and dev.type == "cuda" and fitlib.supported(2 * nq, hidden, k):
        return HipTrainer(nq, device, **kw)
    return DirTrainer(nq, device, **kw)
