"""One densityopt iteration as a single GPU program: no host synchronisation
inside, data parallel over ranks, replayable from a HIP graph.

The reference loop (examples/densityopt/densityopt.py:257-331) per iteration:

1. **D step** -- the discriminator scores the target batch (label 1) and the
   simulated batch (label 0), both losses are back-propagated, and the
   optimizer steps only if ``D_real - D_sim < 0.7`` (two ``.item()`` host
   syncs to decide);
2. **S step** -- unless it is the very first iteration and D was not yet
   separated, the simulation parameters (a LogNormal ``ProbModel``) follow
   the score-function gradient ``mean(log p(theta_i) * (errS_i - b))`` with a
   moving-average baseline ``b`` (one ``.cpu()`` of the per-sample losses);
3. **resample** -- new parameters are drawn and sent to the producers.

:class:`DensityOptStep` runs 1-3 on the device:

* the decisions are device tensors: the D gate feeds ``FusedAdam.step(gate=)``,
  the S gate and the first-iteration flag gate the S optimizer and the
  baseline update with ``torch.where`` -- no ``.item()``;
* with a process group it is data parallel without DDP: D and ProbModel
  gradients live in :class:`~blendtorch.parallel.GradBuckets` and are summed
  in place over RCCL on the compute stream (``1/world`` folded into
  ``FusedAdam``), the gate statistics and the baseline are averaged the same
  way, so every rank takes identical decisions; rank 0's parameter samples
  are broadcast (the reference's ``torch.chunk`` partition of work over
  instances, with one chunk per rank -- densityopt.py:95-107);
* after warm-up iterations the iteration is captured as two HIP graphs and
  replayed: the real-batch half of the D step (it needs only the previous
  iteration's weights: :meth:`prefetch` enqueues it while the producers
  render) and the rest; the caller makes ONE device->host copy per
  iteration: the parameters its producers must render next.

``fused`` (default on the bf16 GPU path): everything between the
discriminator's kernels is two gfx950 kernels (csrc/gpu/dopt.hip) -- the D
statistics and gate (``dopt_gate``), and the whole S step (``dopt_sstep``:
per-sample BCE, the closed-form score-function gradient of the LogNormal
model, gated Adam, baseline, Philox resampling).  The simulated batch is
read in place (one sim-half graph per loader buffer, ``static_inputs``),
the shape ids are read from host-mapped memory and the kernel writes the
rank's samples, the parameters, the statistics and both gates straight into
host-mapped memory (:meth:`host_state`): no device copies in the iteration
and no device->host copy either -- the host waits for the stream and reads.
The fp32 reference path (CPU, ``fused=False``) keeps the PyTorch ProbModel
and autograd; :func:`sstep_reference` is the fused kernel's arithmetic in
PyTorch (tests).

Everything also runs eagerly on the CPU (fp32, gloo) for the test suite.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

__all__ = ['DensityOptStep', 'sstep_reference']


def sstep_reference(logit_s, sid, samples, mean, log_std, b):
    """The fused S step's per-rank means ``[err, g_mu1, g_mu2, g_rho1,
    g_rho2]`` in PyTorch (fp32): ``err_i = -max(log sigmoid(l_i), -100)``
    (BCELoss(reduction='none') against label 1, densityopt.py:290-296) and the
    gradient of ``mean_i(log p(x_sid_i) * (err_i - b))`` w.r.t. the LogNormal
    ``m1m2_mean`` and ``m1m2_log_std`` (densityopt.py:298-300) in closed form
    -- equal to autograd through :class:`~blendtorch.models.ProbModel`
    (tests/test_densityopt.py)."""
    err = -torch.clamp(torch.log(torch.sigmoid(logit_s.float())), min=-100.0)
    x = samples[:, sid]                                   # [2, B]
    d = torch.log(x) - mean[:, None]
    iv = torch.exp(-2.0 * log_std)[:, None]
    w = (err - b)[None, :]
    g_mu = (w * d * iv).mean(1)
    g_rho = (w * (d * d * iv - 1.0)).mean(1)
    return torch.cat([err.mean().reshape(1), g_mu, g_rho])


class DensityOptStep:
    """Params
    ------
    netD: :class:`~blendtorch.models.Discriminator` (64x64, ``adaptive=False``).
    pm: :class:`~blendtorch.models.ProbModel`.
    real: this rank's target batch (model input layout; resident).
    batch: images per rank per iteration (B).
    comm: :class:`~blendtorch.parallel.DeviceComm` for data parallelism, or None.
    bf16: run the discriminator through the bf16 MFMA path
        (``Discriminator.bce_bf16``); inputs must then be bf16 channels-last
        [B, 4, 64, 64] (the first conv ignores the 4th channel).
    graph: capture the iteration in a HIP graph after ``warmup`` eager ones.
    fused: the gate and S step as the gfx950 kernels of csrc/gpu/dopt.hip
        (default: on the bf16 GPU path).
    static_inputs: (fused, graph) sim-half graphs that read the simulated
        batch in place, one per distinct input buffer (a loader with
        ``reuse_buffers=True`` cycles a fixed ring); further buffers are
        copied into a private one.
    seed: the fused sampler's Philox key (default: ``torch.initial_seed()``
        of rank 0, broadcast).
    """

    def __init__(self, netD, pm, real: torch.Tensor, batch: int, comm=None, lr_d=5e-5, betas_d=(0.5, 0.999),
                 lr_s=5e-2, betas_s=(0.7, 0.999), threshold=0.7, alpha=0.9, b0=0.7, bf16=None, graph=True,
                 warmup=2, fused=None, static_inputs=4, seed=None):
        from .. import ops
        from ..parallel import GradBuckets
        self.netD, self.pm, self.comm = netD, pm, comm
        dev = real.device
        self.device = dev
        self.B = int(batch)
        self.world = comm.world if comm is not None else 1
        self.rank = comm.rank if comm is not None else 0
        self.N = self.B * self.world
        self.bf16 = (dev.type == 'cuda') if bf16 is None else bool(bf16)
        self.threshold, self.alpha = float(threshold), float(alpha)
        # the D step's real and sim halves are two backward passes before one update:
        # the sim half's gradients go to second bucket views that optD (FusedAdam) adds
        # in its update kernel -- no AccumulateGrad launch per parameter
        self.gd = GradBuckets(netD.parameters(), second_sinks=True)
        self.gs = GradBuckets(pm.parameters())
        scale = 1.0 / self.world
        self.optD = ops.FusedAdam(netD.parameters(), lr=lr_d, betas=betas_d, grad_scale=scale)
        self.optS = ops.FusedAdam(pm.parameters(), lr=lr_s, betas=betas_s, grad_scale=scale)
        # static state / inputs / outputs (graph-resident)
        self.real = real
        self.sim = torch.empty_like(real)
        self.shape_id = torch.zeros(self.B, dtype=torch.int64, device=dev)
        self.samples = torch.zeros(2, self.N, dtype=torch.float32, device=dev)    # m1, m2 of every rank
        self.b = torch.full((1,), float(b0), device=dev)
        self.first = torch.ones(1, device=dev)
        self.gate_d = torch.ones(1, device=dev)
        self.gate_s = torch.zeros(1, device=dev)
        self.stats = torch.zeros(2, device=dev)         # D_real, D_sim (averaged over ranks)
        self.params_out = torch.zeros(4, device=dev)    # pm.readable_params() after the step
        self.graph_enabled = graph and dev.type == 'cuda'
        self.warmup = int(warmup)
        self.graph = None          # the sim half (the iteration's remainder) once captured
        self.graph_real = None     # the real half
        self._real_done = False    # prefetch() ran the real half of the coming iteration
        self.p_real_mean = torch.zeros(1, device=dev)
        self.iterations = 0
        self.fused = (dev.type == 'cuda' and self.bf16) if fused is None else bool(fused)
        if self.fused:
            if dev.type != 'cuda' or not self.bf16:
                raise ValueError('DensityOptStep(fused=True) needs the bf16 GPU path')
            self._init_fused(lr_s, betas_s, seed, int(static_inputs))

    # -- the fused (gfx950 kernel) path ------------------------------------------------
    def _init_fused(self, lr_s, betas_s, seed, static_inputs):
        import ctypes
        import weakref
        import numpy as np
        from .. import ops
        ext = ops.hip_ext()
        dev = self.device
        for t in (self.pm.m1m2_mean, self.pm.m1m2_log_std):
            if t.dtype != torch.float32 or t.numel() != 2 or not t.is_contiguous() or t.device != dev:
                raise ValueError('DensityOptStep(fused): ProbModel parameters must be contiguous fp32 [2] on the device')
        self._adam = torch.zeros(9, device=dev)              # exp_avg[4], exp_avg_sq[4], step
        self._red = torch.zeros(5, device=dev)
        self._counter = torch.zeros(1, dtype=torch.int32, device=dev)
        nh = 2 * self.B + 8
        hp, hd = ext.host_mapped_alloc(4 * nh)
        sp, sd = ext.host_mapped_alloc(8 * self.B)
        weakref.finalize(self, ext.host_mapped_free, hp)
        weakref.finalize(self, ext.host_mapped_free, sp)
        self._host = torch.from_numpy(np.ctypeslib.as_array((ctypes.c_float * nh).from_address(hp)))
        self._host_sid = np.ctypeslib.as_array((ctypes.c_int64 * self.B).from_address(sp))
        self._host[:] = 0
        self._host_sid[:] = 0
        if seed is None:
            seed = torch.initial_seed()
        seed_t = torch.tensor([int(seed) & 0x7FFFFFFFFFFFFFFF], dtype=torch.int64, device=dev)
        if self.comm is not None:
            self.comm.broadcast_(seed_t, 0)                 # one sampler key: every rank draws the same samples
        self.seed = int(seed_t.item())
        g = self.optS.param_groups[0]
        self._kp = dict(samples=self.samples.data_ptr(), mean=self.pm.m1m2_mean.data_ptr(),
                        log_std=self.pm.m1m2_log_std.data_ptr(), exp_avg=self._adam[0:4].data_ptr(),
                        exp_avg_sq=self._adam[4:8].data_ptr(), adam_step=self._adam[8:9].data_ptr(),
                        lr=float(lr_s), b1=float(betas_s[0]), b2=float(betas_s[1]), eps=float(g['eps']),
                        b=self.b.data_ptr(), first=self.first.data_ptr(), gate_s=self.gate_s.data_ptr(),
                        gate_d=self.gate_d.data_ptr(), stats=self.stats.data_ptr(), alpha=self.alpha,
                        threshold=self.threshold, params_out=self.params_out.data_ptr(), red=self._red.data_ptr(),
                        host=hd, sid=sd, counter=self._counter.data_ptr(), seed=self.seed, B=self.B, N=self.N,
                        rank=self.rank, world=self.world)
        # the D optimizer clears the gradients it reads (also when its gate skips): no zero_() per iteration
        self.optD.set_zero_grads(True)
        self._logit_real = None
        self._keep = None
        self._sims = {}                 # (data_ptr, shape, strides) -> (graph, sim tensor)
        self._static_cap = max(0, static_inputs)
        self._sid_ev = None

    def _ext(self):
        from .. import ops
        return ops.hip_ext(), ops._stream(self.device)

    def _real_half_fused(self):
        # fresh bucket views for this iteration's two backward passes (host flags only: optD
        # clears the gradients it reads): the real half writes the buckets, the sim half the
        # second views optD adds -- no AccumulateGrad launches, in the eager and the captured form
        self.gd.zero_(memset=False)
        loss_r, logits = self.netD.bce_bf16(self.real, 1.0, probs='logits')
        loss_r.backward()
        self._logit_real = logits       # read by the sim half's gate kernel

    def _sim_half_fused(self, sim):
        ext, st = self._ext()
        self.gd.arm_second()   # (each sim-half capture records the second views, not autograd adds)
        loss_s, logit_sim = self.netD.bce_bf16(sim, 0.0, probs='logits')
        loss_s.backward()
        kp = dict(self._kp, logit_real=self._logit_real.data_ptr(), logit_sim=logit_sim.data_ptr())
        if self.comm is None:
            ext.dopt_gate(kp, 0, st)
        else:
            ext.dopt_gate(kp, 1, st)
            self.comm.all_reduce_(self.stats, 'avg')
            ext.dopt_gate(kp, 2, st)
            self.gd.all_reduce(self.comm)
        self.optD.step(gate=self.gate_d)
        with torch.no_grad():
            _, logit_s = self.netD.bce_bf16(sim, 1.0, probs='logits')
        kp['logit_s'] = logit_s.data_ptr()
        if self.comm is None:
            ext.dopt_sstep(kp, 0, st)
        else:
            ext.dopt_sstep(kp, 1, st)
            self.comm.all_reduce_(self._red, 'avg')
            ext.dopt_sstep(kp, 2, st)
        self._keep = (logit_sim, logit_s)

    def host_state(self) -> dict:
        """(fused path) The iteration's results in host-mapped memory, as CPU
        tensor views: this rank's next samples ``[2, B]``, the parameters
        (mu1, mu2, std1, std2), D_real / D_sim and both gates.  Valid once the
        stream has passed the iteration (e.g. ``torch.cuda.current_stream()
        .synchronize()``); the next iteration overwrites them."""
        if not self.fused:
            raise RuntimeError('DensityOptStep.host_state: fused path only')
        B, h = self.B, self._host
        return {'samples': h[:2 * B].view(2, B), 'params': h[2 * B:2 * B + 4], 'stats': h[2 * B + 4:2 * B + 6],
                'gate_d': h[2 * B + 6:2 * B + 7], 'gate_s': h[2 * B + 7:2 * B + 8]}

    def _set_sid(self, shape_id):
        import numpy as np
        sid = shape_id.cpu().numpy() if isinstance(shape_id, torch.Tensor) else np.asarray(shape_id)
        sid = sid.reshape(-1)
        if sid.shape[0] != self.B or (self.B and (int(sid.min()) < 0 or int(sid.max()) >= self.N)):
            raise ValueError(f'DensityOptStep: shape ids must be {self.B} values in [0, {self.N})')
        if self._sid_ev is not None:
            self._sid_ev.synchronize()   # the previous iteration has read them (normally long done)
        self._host_sid[:] = sid

    def _sim_entry(self, sim):
        """The captured sim half that reads ``sim`` in place (captured on first
        use while under the cap), or the copy graph over ``self.sim``."""
        key = (sim.data_ptr(), tuple(sim.shape), tuple(sim.stride()))
        ent = self._sims.get(key)
        if ent is not None:
            return ent
        if len(self._sims) >= self._static_cap:
            ent = self._sims.get('copy')
            if ent is None:
                ent = self._sims['copy'] = self._capture_sim(self.sim)
            self.sim.copy_(sim)
            return ent
        ent = self._sims[key] = self._capture_sim(sim)
        return ent

    def _capture_sim(self, sim):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self.graph_real.pool(), capture_error_mode='thread_local'):
            self._sim_half_fused(sim)
        if self.graph is None:
            self.graph = g
        return (g, sim)

    def _call_fused(self, sim):
        if self.graph_real is not None:
            self.prefetch()
            self._sim_entry(sim)[0].replay()
        elif self.graph_enabled and self.iterations >= self.warmup:
            prev = self._logit_real
            ga = torch.cuda.CUDAGraph()
            with torch.cuda.graph(ga, capture_error_mode='thread_local'):
                self._real_half_fused()
            self.graph_real = ga
            if self._real_done:
                self._logit_real.copy_(prev)      # (once: the real half already ran eagerly this iteration)
            else:
                ga.replay()
                self._real_done = True
            self._sim_entry(sim)[0].replay()
        elif self.graph_enabled:
            self.prefetch()
            self._side(lambda: self._sim_half_fused(sim))
        else:
            self.prefetch()
            self._sim_half_fused(sim)
        ev = torch.cuda.Event()
        ev.record()
        self._sid_ev = ev

    # -- helpers ------------------------------------------------------------------
    def _score(self, x, target):
        """(mean BCE against ``target``, per-sample probabilities)."""
        if self.bf16:
            return self.netD.bce_bf16(x, target)
        out = self.netD(x)
        return F.binary_cross_entropy(out, torch.full_like(out, float(target))), out

    def _avg(self, t):
        if self.comm is not None:
            self.comm.all_reduce_(t, 'avg')
        return t

    def _sample_into(self):
        with torch.no_grad():
            s = self.pm.sample(self.N)
            self.samples[0].copy_(s['m1'])
            self.samples[1].copy_(s['m2'])
            if self.comm is not None:
                self.comm.broadcast_(self.samples, 0)

    # -- the iteration ---------------------------------------------------------------
    def _real_half(self):
        """The D step's target-batch half: forward + backward on the resident
        real batch.  It depends only on the weights the previous iteration
        left, not on the simulated batch, so :meth:`prefetch` can run it while
        the producers still render (reference order kept: real, then sim)."""
        self.gd.zero_()
        loss_r, p_real = self._score(self.real, 1.0)
        loss_r.backward()
        with torch.no_grad():
            self.p_real_mean.copy_(p_real.mean().reshape(1))

    def _sim_half(self):
        # 1. discriminator step (sim half), gated on the device
        loss_s, p_sim = self._score(self.sim, 0.0)
        loss_s.backward()
        with torch.no_grad():
            self.stats.copy_(torch.cat([self.p_real_mean, p_sim.mean().reshape(1)]))
            self._avg(self.stats)
            self.gate_d.copy_((self.stats[0:1] - self.stats[1:2] < self.threshold).float())
        if self.comm is not None:
            self.gd.all_reduce(self.comm)
        self.optD.step(gate=self.gate_d)
        # 2. simulation-parameter step (score-function gradient)
        with torch.no_grad():
            _, p = self._score(self.sim, 1.0)
            err = -torch.clamp(torch.log(p.float()), min=-100.0)     # BCELoss(reduction='none'), target 1
            err_mean = self._avg(err.mean().reshape(1))
            # not the first S step, or D already separates real from sim
            self.gate_s.copy_(torch.clamp((1.0 - self.first) + (1.0 - self.gate_d), max=1.0))
        self.gs.zero_()
        log_probs = self.pm.log_prob({'m1': self.samples[0], 'm2': self.samples[1]})
        loss = (log_probs[self.shape_id] * (err - self.b)).mean()
        loss.backward()
        if self.comm is not None:
            self.gs.all_reduce(self.comm)
        self.optS.step(gate=self.gate_s)
        with torch.no_grad():
            b_new = torch.where(self.first > 0, err_mean, self.alpha * err_mean + (1.0 - self.alpha) * self.b)
            self.b.copy_(torch.where(self.gate_s > 0, b_new, self.b))
            self.first.mul_(1.0 - self.gate_s)
            self.params_out.copy_(self.pm.readable_params())
        # 3. parameters for the next images
        self._sample_into()

    def _iteration(self):
        self._real_half()
        self._sim_half()

    def start(self):
        """Draw the first parameter samples (before any sim batch exists)."""
        if self.fused:
            ext, st = self._ext()
            ext.dopt_sstep(self._kp, 3, st)     # the samples only (and their host-mapped copy)
            return self.samples
        self._sample_into()
        return self.samples

    def _side(self, fn):
        """Warm-up work on a side stream (allocator pools, first-use setup)."""
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            fn()
        torch.cuda.current_stream(self.device).wait_stream(side)

    def prefetch(self):
        """Enqueue the next iteration's real-batch half now (call it after
        sending the parameters, while the producers render): its GPU time
        leaves the critical path between the sim batch's arrival and the
        next parameters.  Optional -- :meth:`__call__` runs it otherwise."""
        if self._real_done:
            return
        half = self._real_half_fused if self.fused else self._real_half
        if self.graph_real is not None:
            self.graph_real.replay()
        elif self.graph_enabled:
            self._side(half)
        else:
            half()
        self._real_done = True

    def __call__(self, sim: torch.Tensor, shape_id: torch.Tensor):
        """One iteration on a simulated batch and its global sample ids.
        Returns the device tensor of the next samples ([2, N]: m1, m2)."""
        if tuple(sim.shape) != tuple(self.sim.shape) or sim.dtype != self.sim.dtype:
            raise ValueError(f'DensityOptStep: sim batch {sim.dtype} {tuple(sim.shape)}, expected '
                             f'{self.sim.dtype} {tuple(self.sim.shape)}')
        if self.fused:
            self._set_sid(shape_id)
            self._call_fused(sim)
            self._real_done = False
            self.iterations += 1
            return self.samples
        self.sim.copy_(sim)
        self.shape_id.copy_(shape_id, non_blocking=True)
        if self.graph is not None:
            self.prefetch()
            self.graph.replay()
        elif self.graph_enabled and self.iterations >= self.warmup:
            self._capture_and_replay()
        elif self.graph_enabled:
            self.prefetch()
            self._side(self._sim_half)
        else:
            self.prefetch()
            self._sim_half()
        self._real_done = False
        self.iterations += 1
        return self.samples

    def _capture_and_replay(self):
        # capture records without running: each half then runs as its first replay
        # (the real half only if prefetch() has not run it for this iteration).
        # thread_local: the stream loader's worker thread keeps making HIP calls
        ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(ga, capture_error_mode='thread_local'):
            self._real_half()
        with torch.cuda.graph(gb, pool=ga.pool(), capture_error_mode='thread_local'):
            self._sim_half()
        self.graph_real, self.graph = ga, gb
        if not self._real_done:
            ga.replay()
        gb.replay()

    def my_samples(self, samples: Optional[torch.Tensor] = None):
        """This rank's chunk of the samples ([2, B]) and their global ids."""
        s = self.samples if samples is None else samples
        lo = self.rank * self.B
        return s[:, lo:lo + self.B], torch.arange(lo, lo + self.B)
