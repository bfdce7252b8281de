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

Everything also runs eagerly on the CPU (fp32, gloo) for the test suite.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

__all__ = ['DensityOptStep']


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
    """

    def __init__(self, netD, pm, real: torch.Tensor, batch: int, comm=None, lr_d=5e-5, betas_d=(0.5, 0.999),
                 lr_s=5e-2, betas_s=(0.7, 0.999), threshold=0.7, alpha=0.9, b0=0.7, bf16=None, graph=True,
                 warmup=2):
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
        self.gd = GradBuckets(netD.parameters())
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
        if self.graph is not None:
            self.graph_real.replay()
        elif self.graph_enabled:
            self._side(self._real_half)
        else:
            self._real_half()
        self._real_done = True

    def __call__(self, sim: torch.Tensor, shape_id: torch.Tensor):
        """One iteration on a simulated batch and its global sample ids.
        Returns the device tensor of the next samples ([2, N]: m1, m2)."""
        if tuple(sim.shape) != tuple(self.sim.shape) or sim.dtype != self.sim.dtype:
            raise ValueError(f'DensityOptStep: sim batch {sim.dtype} {tuple(sim.shape)}, expected '
                             f'{self.sim.dtype} {tuple(self.sim.shape)}')
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
