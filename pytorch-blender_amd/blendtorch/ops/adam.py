"""Adam / AdamW for the consumer step as two gfx950 launches per parameter group.

``torch.optim.Adam(fused=True, capturable=True)`` on ROCm spends ~50 us per
DCGAN-discriminator step in two multi-tensor-apply kernels that put only a
few dozen workgroups on a 256-CU chip (profiles/r2/disc_mtrace_kernels.txt).
Here one single-lane kernel advances the step counter and the bias
corrections on the device (``adam_schedule``), and one kernel updates every
parameter of the group, one lane per four elements across all tensors
(``adam_update``: a 0.7 M-parameter model is ~700 workgroups).  Both read
their scalars from device memory, so the pair is capturable in a HIP graph
and replays correctly; ``set_lr`` changes the learning rate of a captured
optimizer (it writes the device copy the schedule kernel reads).

Optional ``bf16_shadow``: the update also writes a bf16 copy of every new
weight (``shadow(p)``), which a bf16 forward can read instead of casting the
fp32 master weights on every step.  :meth:`FusedAdam.enable_conv_shadows`
adds, for 4x4 convolution weights, the transposed bf16 copy a data-gradient
kernel reads (``shadow_t(p)``, ``conv_weights_t`` layout) -- the consumer
step's per-step cast and transpose launches then disappear.

``one_launch=True`` (or ``BT_ADAM_ONE_LAUNCH=1``): where a group fits one
launch (<= 32 tensors) there is no ``adam_schedule`` launch.  The schedule of
the coming step is worked out AHEAD -- once when the group's device state is
made (and after ``set_lr`` / ``set_grad_scale``), then by the block of each
update that takes the last ticket, which also advances the counter -- so the
update's blocks only read it.  (Round 3's one-launch form had every block work
the schedule out itself: one lane's fp64 powers behind a barrier, 3.7 us
slower than two launches on the bench discriminator, scripts/adam_bench.py.)
:meth:`set_zero_grads` makes the update clear each gradient after reading it,
so persistent gradient buffers (``parallel.GradBuckets``) need no zero-fill
launch before the next backward.

Data parallel: ``grad_scale`` multiplies every gradient inside the update
kernel, so a summing all-reduce of the gradients (``parallel.GradBuckets``)
needs no separate ``div_`` by the world size.  ``step(gate=t)`` takes a device
scalar: where ``t == 0`` the step is a no-op (counter, moments and weights
untouched) -- a conditional optimizer step without a host synchronisation,
capturable in a graph (densityopt's ``D_real - D_sim < 0.7`` rule).

Arithmetic is PyTorch's Adam (torch/optim/adam.py, non-amsgrad): L2 weight
decay added to the gradient, or decoupled (AdamW) when ``decoupled=True``.
CPU tensors run the same formulas in PyTorch (reference path and tests).
The reference trains with ``torch.optim.Adam`` on the CPU-collated batches
(examples/densityopt/densityopt.py:270-274).
"""
from __future__ import annotations

import torch

from . import _count, _dense, _stream, hip_ext


def _second_grad(p):
    """The second gradient contribution of this step held in ``p``'s second
    bucket view (:class:`~blendtorch.parallel.GradBuckets` ``second_sinks``),
    or None."""
    if getattr(p, '_bt_grad_second', False) and p.grad is getattr(p, '_bt_grad_sink', None):
        return p._bt_grad_sink2
    return None

__all__ = ['FusedAdam']

import os  # noqa: E402

_ONE_LAUNCH_DEFAULT = os.environ.get('BT_ADAM_ONE_LAUNCH', '0') == '1'
# the schedule handed to the backward's last slice-reduce launch by CapturedStep (BT_ADAM_ATTACH=0: its own launch)
_ATTACH = os.environ.get('BT_ADAM_ATTACH', '1') not in ('', '0')

_MAX_PER_LAUNCH = 32   # kMaxAdam (csrc/gpu/kernels.h)
# the backward's last weight-gradient slice reduce summed inside the update launch (attach_reduce;
# BT_ADAM_FUSE_REDUCE=0: its own launch)
_FUSE_REDUCE = os.environ.get('BT_ADAM_FUSE_REDUCE', '1') not in ('', '0')


def _ops():
    import sys
    return sys.modules[__package__]


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, decoupled=False,
                 maximize=False, bf16_shadow=False, grad_scale=1.0, one_launch=None):
        if lr < 0 or eps < 0 or weight_decay < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError(f'invalid Adam hyper-parameters lr={lr} betas={betas} eps={eps} wd={weight_decay}')
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, decoupled=decoupled,
                        maximize=maximize, bf16_shadow=bf16_shadow)
        super().__init__(params, defaults)
        self._grad_scale = float(grad_scale)
        # id(group) -> device scalars (kept out of param_groups / state_dict).
        # Each entry holds its group, so an id cannot be reused while it lives.
        self._dev = {}
        self._zero_grads = False
        self._one_launch = _ONE_LAUNCH_DEFAULT if one_launch is None else bool(one_launch)
        self._attached = None   # (group id, lr) of a schedule handed to the backward (attach_schedule)

    # -- per-group device scalars ------------------------------------------
    def _group_state(self, group):
        dev = group['params'][0].device
        gs = self._dev.get(id(group))
        if gs is None or gs['group'] is not group or gs['step'].device != dev:
            # a loaded state_dict carries the counter as each parameter's 'step'
            prev = next((self.state[p]['step'] for p in group['params'] if 'step' in self.state.get(p, {})), None)
            step = torch.zeros(1, dtype=torch.float32, device=dev)
            if prev is not None:
                step.fill_(float(prev.reshape(-1)[0]))
            gs = {'step': step, 'group': group,
                  'hp': torch.tensor([float(group['lr']), self._grad_scale], dtype=torch.float32, device=dev),
                  'sched': torch.zeros(5, dtype=torch.float32, device=dev),
                  'ticket': torch.zeros(4, dtype=torch.int32, device=dev),
                  'lr': float(group['lr']), 'grad_scale': self._grad_scale}
            self._dev[id(group)] = gs
            self._prime(group, gs)
            for p in group['params']:
                if self.state.get(p):
                    self.state[p]['step'] = step
        return gs

    def _prime(self, group, gs):
        """One-launch form: work out the coming step's schedule now (the
        counter, lr or gradient scale changed outside an update)."""
        if self._one_launch and gs['step'].is_cuda:
            b1, b2 = group['betas']
            hip_ext().adam_schedule_prime(gs['step'].data_ptr(), gs['hp'].data_ptr(), gs['sched'].data_ptr(),
                                          b1, b2, _stream(gs['step'].device))

    def attach_schedule(self):
        """Hand this step's schedule (the step counter and bias corrections)
        to the next weight-gradient slice-reduce launch of the backward about to
        run (its first lane computes it): the update then needs no schedule
        launch.  Call right before the backward, then :meth:`step` without a
        gate; a backward without such a launch leaves the job to :meth:`step`.
        Only for one GPU parameter group outside the one-launch form; returns
        whether it attached."""
        self._attached = None
        if not _ATTACH or self._one_launch:
            return False
        groups = [g for g in self.param_groups if g['params']]
        if len(groups) != 1 or not groups[0]['params'][0].is_cuda:
            return False
        group = groups[0]
        gs = self._group_state(group)
        if gs['lr'] != float(group['lr']):
            if torch.cuda.is_current_stream_capturing():
                return False
            gs['hp'][0].fill_(float(group['lr']))
            gs['lr'] = float(group['lr'])
        b1, b2 = group['betas']
        dev = gs['step'].device
        hip_ext().adam_attach_schedule(gs['step'].data_ptr(), gs['hp'].data_ptr(), gs['sched'].data_ptr(), b1, b2,
                                       dev.index if dev.index is not None else torch.cuda.current_device(),
                                       _stream(dev))
        self._attached = (id(group), gs['lr'], gs)
        return True

    def attach_reduce(self):
        """Let the update take the backward's last weight-gradient slice
        reduce (the ordered one of a 4x4 convolution weight whose gradient is
        written into its bucket view, ``parallel.GradBuckets``): the reduce is
        not launched but summed by extra blocks of the update launch, which also
        write the gradient (0 under :meth:`set_zero_grads`) -- one launch fewer
        per step.  Call right before a backward that no collective follows,
        then :meth:`step`; :meth:`detach_reduce` runs a reduce no update took.
        One GPU parameter group outside the one-launch form; returns whether it
        attached."""
        if not _FUSE_REDUCE or self._one_launch:
            return False
        groups = [g for g in self.param_groups if g['params']]
        if len(groups) != 1 or not groups[0]['params'][0].is_cuda:
            return False
        ops = _ops()
        ops._claim_flush()
        ops._REDUCE_CLAIM = {'params': {id(p) for p in groups[0]['params']}, 'got': None}
        return True

    def detach_reduce(self):
        """Run a slice reduce :meth:`attach_reduce` let the backward hand over
        that no update took (e.g. the backward raised), and stop taking them."""
        ops = _ops()
        ops._claim_flush()
        ops._REDUCE_CLAIM = None

    def detach_schedule(self):
        """Drop a schedule :meth:`attach_schedule` handed out (e.g. the
        backward raised).  If a slice-reduce launch already ran it, the device
        counter has advanced for an update that will not happen: step it back,
        so the next update's bias correction is the right one."""
        if self._attached is not None:
            ext = hip_ext()
            taken = bool(ext.adam_schedule_taken())
            ext.adam_detach_schedule()
            if taken:
                self._attached[2]['step'].sub_(1.0)
            self._attached = None

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._dev.clear()     # the loaded groups are new dicts: rebuild their counters from the state

    @property
    def grad_scale(self):
        return self._grad_scale

    def set_grad_scale(self, scale):
        """Factor every gradient is multiplied by in the update (e.g.
        ``1 / world_size`` after a summing all-reduce); also for a captured
        optimizer (the device copy is rewritten)."""
        self._grad_scale = float(scale)
        for gs in self._dev.values():
            gs['hp'][1].fill_(self._grad_scale)
            gs['grad_scale'] = self._grad_scale
            self._prime(gs['group'], gs)

    def set_lr(self, lr, group=0):
        """Change the learning rate, also for an optimizer captured in a graph."""
        g = self.param_groups[group]
        g['lr'] = float(lr)
        gs = self._group_state(g)
        gs['hp'][0].fill_(float(lr))
        gs['lr'] = float(lr)
        self._prime(g, gs)

    def _state(self, p, group):
        st = self.state[p]
        if 'exp_avg' not in st:
            st['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
        for k in ('exp_avg', 'exp_avg_sq'):
            if st[k].stride() != p.stride() or st[k].device != p.device:   # e.g. loaded from a state_dict
                st[k] = torch.empty_like(p).copy_(st[k])
        st['step'] = self._group_state(group)['step']              # one counter per group
        if group['bf16_shadow'] and 'shadow' not in st:
            st['shadow'] = p.detach().to(torch.bfloat16)
        return st

    def shadow(self, p):
        """The bf16 copy of ``p`` the last update wrote (``bf16_shadow=True``
        or :meth:`enable_conv_shadows`)."""
        return self.state[p]['shadow']

    def shadow_t(self, p):
        """The transposed bf16 copy of conv weight ``p`` (:meth:`enable_conv_shadows`)."""
        return self.state[p]['shadow_t']

    def enable_conv_shadows(self, weights, transpose=None):
        """Keep, for each fp32 4x4 convolution weight in ``weights`` (channels-
        last [Cout, Cin, 4, 4], on the GPU), a bf16 copy and -- where
        ``transpose[i]`` (default: Cout and Cin multiples of 32) -- its data-gradient
        transpose up to date: made now from the current weights and rewritten
        by every update.  A weight changed outside this optimizer (e.g. a
        model ``load_state_dict``) needs :meth:`refresh_shadows`."""
        from . import conv_weights_t
        found = {id(p) for g in self.param_groups for p in g['params']}
        weights = list(weights)
        if transpose is None:
            transpose = [int(p.shape[0]) % 32 == 0 and int(p.shape[1]) % 32 == 0 for p in weights]
        for p, tr in zip(weights, transpose):
            if id(p) not in found:
                raise ValueError('enable_conv_shadows: a weight is not a parameter of this optimizer')
            if not (p.is_cuda and p.dtype == torch.float32 and p.dim() == 4 and tuple(p.shape[2:]) == (4, 4)
                    and p.is_contiguous(memory_format=torch.channels_last)):
                raise ValueError('enable_conv_shadows: needs channels-last fp32 [Cout, Cin, 4, 4] GPU weights')
            if tr and (int(p.shape[0]) % 32 or int(p.shape[1]) % 32):
                raise ValueError('enable_conv_shadows: a transposed shadow needs Cout % 32 == Cin % 32 == 0')
            st = self.state[p]
            st['shadow'] = p.detach().to(torch.bfloat16)
            if tr:
                st['shadow_t'] = conv_weights_t([st['shadow']])[0]
            else:
                st.pop('shadow_t', None)

    def refresh_shadows(self):
        """Rewrite every bf16 shadow from the current fp32 weights."""
        from . import conv_weights_t
        for g in self.param_groups:
            for p in g['params']:
                st = self.state.get(p, {})
                if 'shadow' in st:
                    st['shadow'].copy_(p.detach())
                if 'shadow_t' in st:
                    st['shadow_t'].copy_(conv_weights_t([st['shadow']])[0])

    def set_zero_grads(self, on=True):
        """Clear every (fp32) gradient inside the update kernel after reading
        it, also when a gate skips the step."""
        self._zero_grads = bool(on)

    # -- step -----------------------------------------------------------------
    @torch.no_grad()
    def step(self, closure=None, gate=None):
        """One update; ``gate`` (optional 1-element float tensor on the
        parameters' device): skip the step where it is 0."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            params = [p for p in group['params'] if p.grad is not None]
            if not params:
                continue
            gs = self._group_state(group)
            capturing = params[0].is_cuda and torch.cuda.is_current_stream_capturing()
            if gs['lr'] != float(group['lr']) and not capturing:
                gs['hp'][0].fill_(float(group['lr']))   # lr edited through param_groups
                gs['lr'] = float(group['lr'])
                self._prime(group, gs)
            states = [self._state(p, group) for p in params]
            if gate is not None and (gate.numel() != 1 or gate.device != params[0].device):
                raise ValueError('FusedAdam.step: gate must be a 1-element tensor on the parameters\' device')
            if params[0].is_cuda:
                self._step_gpu(group, gs, params, states, gate)
            else:
                self._step_reference(group, gs, params, states, gate)
                if self._zero_grads:
                    for p in params:
                        p.grad.zero_()
                        if _second_grad(p) is not None:
                            _second_grad(p).zero_()
        return loss

    def _step_gpu(self, group, gs, params, states, gate=None):
        ext = hip_ext()
        b1, b2 = group['betas']
        stream = _stream(params[0].device)
        for p in params:
            # elementwise update: any dense layout works as long as p, grad,
            # exp_avg and exp_avg_sq share it (the state is allocated like p)
            if p.dtype != torch.float32 or not _dense(p):
                raise ValueError('FusedAdam (GPU) needs dense fp32 parameters (contiguous or channels-last)')
        if gate is not None and gate.dtype != torch.float32:
            raise ValueError('FusedAdam.step: gate must be float32 on the GPU')
        one = self._one_launch and len(params) <= _MAX_PER_LAUNCH
        att, self._attached = getattr(self, '_attached', None), None
        taken = att is not None and att[0] == id(group) and bool(ext.adam_schedule_taken())
        if att is not None:
            ext.adam_detach_schedule()
        if taken:
            # a slice-reduce launch of the backward already advanced the counter and
            # wrote this step's schedule (attach_schedule)
            if gate is not None:
                raise RuntimeError('FusedAdam.step: a gate after attach_schedule (the schedule already ran ungated)')
            _count('adam_schedule_attached')
            if gs['lr'] != att[1]:   # lr edited after the attach: this step's schedule again, counter as is
                ext.adam_schedule_prime(gs['step'].data_ptr(), gs['hp'].data_ptr(), gs['sched'].data_ptr(), b1, b2,
                                        stream, 0.0)
        elif not one:
            _count('adam_schedule')
            ext.adam_schedule(gs['step'].data_ptr(), gs['hp'].data_ptr(), gs['sched'].data_ptr(), b1, b2, stream,
                              gate.data_ptr() if gate is not None else 0)
        zero = self._zero_grads and all(p.grad.dtype == torch.float32 for p in params)
        # a slice reduce the backward handed over (attach_reduce): its weight leaves the lists and
        # extra blocks of the first launch sum its gradient and update it (AdamParams::fr)
        ops = _ops()
        claim, fr = ops._REDUCE_CLAIM, None
        if claim is not None and claim['got'] is not None:
            res, keep, fp, _dev = claim['got']
            k = next((i for i, p in enumerate(params) if p is fp), -1)
            st = states[k] if k >= 0 else None
            if (k >= 0 and not one and fp.grad is keep[1] and fp.grad.dtype == torch.float32
                    and fp.grad.stride() == fp.stride() and _second_grad(fp) is None and 'shadow_t' not in st):
                claim['got'] = None
                fr = (res, [fp.grad.data_ptr(), fp.data_ptr(), st['exp_avg'].data_ptr(), st['exp_avg_sq'].data_ptr(),
                            st['shadow'].data_ptr() if 'shadow' in st else 0], keep)
                params, states = params[:k] + params[k + 1:], states[:k] + states[k + 1:]
                _count('adam_fused_reduce')
            else:
                ops._claim_flush()   # the gradient first, then the plain update reads it
        for i in range(0, max(len(params), 1 if fr is not None else 0), _MAX_PER_LAUNCH):
            ps, ss = params[i:i + _MAX_PER_LAUNCH], states[i:i + _MAX_PER_LAUNCH]
            grads = []
            for p in ps:
                g = p.grad
                if g.dtype not in (torch.float32, torch.bfloat16) or g.dtype != ps[0].grad.dtype:
                    raise ValueError('FusedAdam: gradients must all be fp32 or all bf16')
                if g.stride() != p.stride():
                    g = torch.empty_like(p, dtype=g.dtype).copy_(g)   # same memory order as the parameter
                grads.append(g)
            _count('adam_update')
            trans = any('shadow_t' in s for s in ss)
            # a second contribution of this step (a second backward pass) sits in the
            # parameter's second bucket view (GradBuckets(second_sinks=True)): the update
            # kernel adds it, instead of an AccumulateGrad launch per parameter
            g2 = [_second_grad(p) for p in ps]
            if any(x is not None for x in g2) and grads and grads[0].dtype != torch.float32:
                raise ValueError('FusedAdam: second gradient contributions need fp32 gradients')
            ext.adam_update([p.data_ptr() for p in ps], [g.data_ptr() for g in grads],
                            [s['exp_avg'].data_ptr() for s in ss], [s['exp_avg_sq'].data_ptr() for s in ss],
                            [s['shadow'].data_ptr() if 'shadow' in s else 0 for s in ss],
                            [p.numel() for p in ps], gs['sched'].data_ptr(),
                            int(bool(grads) and grads[0].dtype == torch.bfloat16),
                            b1, b2, group['eps'], group['weight_decay'], int(group['decoupled']),
                            int(group['maximize']), stream,
                            step=gs['step'].data_ptr() if one else 0, hp=gs['hp'].data_ptr() if one else 0,
                            gate=gate.data_ptr() if (one and gate is not None) else 0,
                            ticket=gs['ticket'].data_ptr() if one else 0, zero_grad=int(zero),
                            shadow_t=[s['shadow_t'].data_ptr() if 'shadow_t' in s else 0 for s in ss] if trans else [],
                            tcout=[int(p.shape[0]) if 'shadow_t' in s else 0 for p, s in zip(ps, ss)] if trans else [],
                            tcin=[int(p.shape[1]) if 'shadow_t' in s else 0 for p, s in zip(ps, ss)] if trans else [],
                            grads2=[x.data_ptr() if x is not None else 0 for x in g2]
                            if any(x is not None for x in g2) else [],
                            fused_reduce=fr[0] if (fr is not None and i == 0) else None,
                            fr_tensors=fr[1] if (fr is not None and i == 0) else [])
            if zero:
                for p, g in zip(ps, grads):
                    if g is not p.grad:      # a re-strided copy was read and cleared: clear the real one
                        p.grad.zero_()

    @staticmethod
    def _step_reference(group, gs, params, states, gate=None):
        """fp32 PyTorch reference of the same update (CPU tensors)."""
        if gate is not None and float(gate.reshape(-1)[0]) == 0.0:
            return
        b1, b2 = group['betas']
        gs['step'] += 1
        s = float(gs['step'])
        lr, wd = float(gs['hp'][0]), group['weight_decay']
        step_size = lr / (1 - b1 ** s)
        inv_bc2 = 1.0 / (1 - b2 ** s) ** 0.5
        scale = float(gs['hp'][1])
        for p, st in zip(params, states):
            g = p.grad.float()
            g2 = _second_grad(p)
            if g2 is not None:
                g = g + g2
            if scale != 1.0:
                g = g * scale
            if group['maximize']:
                g = -g
            if wd:
                if group['decoupled']:
                    p.mul_(1 - lr * wd)
                else:
                    g = g + wd * p
            st['exp_avg'].mul_(b1).add_(g, alpha=1 - b1)
            st['exp_avg_sq'].mul_(b2).addcmul_(g, g, value=1 - b2)
            p.addcdiv_(st['exp_avg'], st['exp_avg_sq'].sqrt().mul_(inv_bc2).add_(group['eps']), value=-step_size)
            if 'shadow' in st:
                st['shadow'].copy_(p)
            if 'shadow_t' in st:
                from . import conv_weights_t
                st['shadow_t'].copy_(conv_weights_t([st['shadow']])[0])
