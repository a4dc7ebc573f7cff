"""One PPO/ROA minibatch (reference rsl_rl ppo.py:186-276) on the S8 GEMM core (include/lgx_s8.h).

The GPU update's minibatch as a fixed kernel sequence over preallocated buffers — no autograd
graph, no per-call allocation (the hipGraph captures exactly these launches):

  per update   the network inputs of every row, gathered in the epoch-shared permutation
               (rollout_storage.py:141-147) and split into S8 (bf16 hi/lo planes) in one launch
  per minibatch
    1  the 17 weight matrices -> S8 (one launch; they change after every Adam step) — at the
       update's first minibatch only: the optimizer tail (lgx_ppo_tail's Adam launch) writes the
       updated weights' S8 copies itself (tail_table)
    2  forward, one grouped launch per level: {priv, scan, est, critic} layers 0..2, then the
       critic's last layer beside the actor's first, then the actor (actor_critic.py:82-107,
       support_networks.py:25-80). Every epilogue writes its output in S8 (the next GEMMs'
       operand) — the encoders' last layers straight into their columns of the actor input —
       and in fp32 where a loss reads it (mu, V(s), the privileged latent, the estimate)
    3  loss heads forward + backward in one launch (lgx_loss_heads_fused: surrogate, clipped
       value loss, entropy, KL, ROA regulariser, estimator loss; ppo.py:196-262), which also
       writes the narrow output gradients in S8 with their column sums (the last layers' bias
       gradients)
    4  input gradients, one grouped launch per level back through the chains; each epilogue
       applies ELU'(y) of the layer below (from its S8 output), writes S8, and sums its columns
       per 128-row tile (that layer's bias gradient). The actor's first layer forms the gradient
       of its latent columns only (the inputs that carry one), plus the regulariser's gradient
       of the privileged latent (the two paths autograd would sum)
    5  every weight gradient in ONE split-K launch, then one reduction launch into the flat
       gradient buffer (weights, from the split partials; biases, from the column-sum partials)

The actor input lives in S8 in a segmented layout: [obs | priv latent | scan latent | est], each
part starting at a multiple of 8 columns (an S8 group), so the encoders write and read their
parts as whole groups; the actor's first-layer weights are split into the same layout.

Numerics: the GEMMs are the same 3 x bf16 products as lgx_mlp.h (identical hi/lo of the same
fp32 values); ELU' reads y as hi + lo (~2^-17 relative of y), the bias gradients are summed per
tile then over tiles (a different fixed order): within the stated fp32 tolerances of the update
(tests/test_gpu_s8_update.py), not bit-identical to the autograd path.
"""
import os

import torch

from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H
from legged_gym_custom_amd.rsl_rl.modules import hip_s8 as S

ENC_CHAIN = os.environ.get("LGX_S8_CHAIN", "1") != "0"  # the encoders' forward as one chain launch
# the actor's / critic's last layers fused around the PPO head (lgx_loss_heads_tail)
HEADS_TAIL = os.environ.get("LGX_HEADS_TAIL", "1") != "0"
ROW_ALIGN = 64  # minibatch rows: whole K steps of every weight-gradient chunk


def _chain(mod):
    c = mod._chain() if isinstance(mod, H.HipMLP) else None
    if c is None:
        return None
    layers, flags = c
    if flags[-1] or not all(flags[:-1]):
        return None  # [Linear, ELU]* Linear only
    return layers


class _Part:
    """One chain's buffers and launch arguments."""

    def __init__(self, name, layers):
        self.name = name
        self.layers = layers                       # nn.Linear list
        self.W = [m.weight for m in layers]
        self.b = [m.bias for m in layers]
        self.n = len(layers)


class S8Minibatch:
    @staticmethod
    def supported(alg, mb):
        if not alg.on_gpu or mb % ROW_ALIGN or mb <= 0:
            return False
        # no fallback for a broken build: with the S8 update selected (LGX_S8_UPDATE, default on)
        # a missing or stale liblgx_s8.so raises here (S.lib), it never silently selects the
        # autograd path; only shapes the S8 layout does not cover return False
        S.lib()
        ac = alg.actor_critic
        chains = [_chain(ac.actor), _chain(ac.critic), _chain(ac.privileged_encoder_.priv_encoder),
                  _chain(ac.scan_encoder.scan_encoder), _chain(alg.estimator.estimator)]
        if any(c is None for c in chains):
            return False
        if sum(len(c) for c in chains) > S.GROUP_MAX:  # one weight-gradient group (lgx_s8_pick_split)
            return False
        if ac.num_scan_obs <= 0 or ac.num_privileged_obs <= 0:
            return False
        est = alg.estimator
        c0 = 0 if est.use_history else ac.num_proprio * ac.history_buffer_length
        if c0 % 8:
            return False
        return len(chains[0]) >= 2

    def __init__(self, alg, rows, mb):
        ac = alg.actor_critic
        self.alg, self.rows, self.mb = alg, rows, mb
        dev = alg.device
        self.dev = dev
        self.actor = _Part("actor", _chain(ac.actor))
        self.critic = _Part("critic", _chain(ac.critic))
        self.priv = _Part("priv", _chain(ac.privileged_encoder_.priv_encoder))
        self.scan = _Part("scan", _chain(ac.scan_encoder.scan_encoder))
        self.est = _Part("est", _chain(alg.estimator.estimator))
        self.parts = [self.priv, self.scan, self.est, self.critic, self.actor]
        # the actor input's logical columns and their S8 positions
        self.nobs = ac.num_proprio * (1 + ac.history_buffer_length)
        self.nlat = self.priv.W[-1].shape[0]
        self.nscan = self.scan.W[-1].shape[0]
        self.nest = ac.num_estimated_obs
        if self.actor.W[0].shape[1] != self.nobs + self.nlat + self.nscan + self.nest:
            raise ValueError("actor input width does not match [obs | latent | scan latent | est]")
        r8 = lambda x: (x + 7) // 8 * 8  # noqa: E731
        self.P0 = r8(self.nobs)
        self.P1 = self.P0 + r8(self.nlat)
        self.P2 = self.P1 + r8(self.nscan)
        self.W8 = self.P2 + r8(self.nest)
        self.spans = [(0, 0, self.nobs), (self.nobs, self.P0, self.nlat), (self.nobs + self.nlat, self.P1, self.nscan),
                      (self.nobs + self.nlat + self.nscan, self.P2, self.nest)]  # (logical col, S8 col, width)
        est = alg.estimator
        self.est_c0 = 0 if est.use_history else self.nobs - ac.num_proprio
        self.est_k = self.est.W[0].shape[1]
        # ---- per-update inputs (all rows, permuted)
        # (one spare block of rows: a weight-gradient read of a column span that starts past column
        # 0 may run up to that offset past the end of a row)
        self.ain = S.empty(rows + ROW_ALIGN, self.W8, dev)
        self.crin = S.empty(rows + ROW_ALIGN, self.critic.W[0].shape[1], dev)
        self.prin = S.empty(rows + ROW_ALIGN, self.priv.W[0].shape[1], dev)
        self.scin = S.empty(rows + ROW_ALIGN, self.scan.W[0].shape[1], dev)
        # ---- weights in S8 (actor layer 0 in the segmented layout)
        for p in self.parts:
            p.Ws = [S.empty(W.shape[0], (self.W8 if (p is self.actor and l == 0) else W.shape[1]), dev)
                    for l, W in enumerate(p.W)]
        # ---- activations (S8) of every hidden layer; fp32 where a loss reads them
        for p in self.parts:
            p.out = [S.empty(mb, W.shape[0], dev) for W in p.W[:-1]]
        self.mu = torch.empty(mb, self.actor.W[-1].shape[0], device=dev)
        self.value = torch.empty(mb, 1, device=dev)
        self.pred = torch.empty(mb, self.est.W[-1].shape[0], device=dev)
        self.lat = torch.empty(mb, self.nlat, device=dev)
        # ---- output gradients (S8) of every layer: dy[l] = dL/d(output of layer l)
        for p in self.parts:
            p.dy = [S.empty(mb, W.shape[0], dev) for W in p.W]
        # the encoders' last-layer output gradients: one buffer, the actor-input layout's latent
        # part (priv at 0, scan at P1 - P0), written by the actor's first input-gradient launch
        self.dlat = S.empty(mb, self.W8 - self.P0, dev)
        self.priv.dy[-1] = None
        self.scan.dy[-1] = None
        # the regulariser's gradient of the privileged latent (fp32: the addend of the actor's
        # latent-column input gradient) and the loss heads' partial-sum workspaces
        self.dp = torch.empty(mb, self.nlat, device=dev)
        # the actor's / critic's last layers inside the loss-heads launch (lgx_loss_heads_tail):
        # their forward, the PPO head and their input gradients in one launch (replacing the
        # last forward level, lgx_loss_heads_fused and the first input-gradient level)
        Wa, Wc = self.actor.W[-1], self.critic.W[-1]
        self.tail = (HEADS_TAIL and self.actor.n >= 2 and self.critic.n >= 2 and Wa.shape[0] <= 16 and Wc.shape[0] == 1
                     and all(W.shape[1] % 8 == 0 and 8 <= W.shape[1] <= 256 and W.is_contiguous() for W in (Wa, Wc)))
        self.ntail = (mb + H.HEADS_TAIL_ROWS - 1) // H.HEADS_TAIL_ROWS
        self.head_ws = torch.empty(19 * max(self.ntail, (mb + 63) // 64), device=dev)
        self.aux_ws = torch.empty(2 * ((mb + 63) // 64), device=dev)
        # ---- weight-gradient split-K workspace and bias-gradient partials
        shapes = []
        for p in self.parts:
            for l, W in enumerate(p.W):
                n_in = self.W8 if (p is self.actor and l == 0) else W.shape[1]
                shapes.append((W.shape[0], n_in, mb))
        self.splits = S.pick_split(shapes)
        tot = sum(s * m * n for s, (m, n, _k) in zip(self.splits, shapes))
        self.dw_ws = torch.empty(tot, device=dev)
        self.tiles_m = (mb + S.TILE_M - 1) // S.TILE_M  # column-sum partials of the FWD / DX epilogues
        self.nsb = (mb + S.SPLIT_ROWS - 1) // S.SPLIT_ROWS
        for p in self.parts:
            # colsum partials of dy[l] (the bias gradient of layer l): [tiles][out_l] (the
            # heads-tail launch: one per 32-row block for the last two layers of actor / critic)
            p.cs = [torch.empty(max(self.tiles_m, self.nsb, self.ntail), W.shape[0], device=dev) for W in p.W]
        self.cs_lat = torch.empty(self.tiles_m, self.P2 - self.P0, device=dev)
        # launch schedule: the level (grouped launch) of each chain's layer is its depth plus this
        # shift — the critic and the estimator do not feed the actor, so they can share the
        # actor's under-filled levels instead of running ahead of it (forward / input gradients)
        # (measured on go2 at 24,576-row minibatches, tools/s8_levels.py: 765 -> 734 us per minibatch)
        self.fwd_shift = {"critic": 3, "est": 3}
        self.dx_shift = {"critic": 0, "est": 2}
        # a first layer as column slices over the levels before its own (measured for the
        # critic beside the privileged / scan encoders' narrow levels: 2 / 3 / 4 slices 720 / 746
        # / 739 us per minibatch against 710 unsliced — not used)
        self.l0_slices = {"critic": 1}
        # the privileged and scan encoders' forward as one chain launch (lgx_s8_chain)
        # instead of their own three grouped levels
        self.enc_chain = ENC_CHAIN and all(p.n <= S.CHAIN_MAXL and max(max(W.shape) for W in p.W) <= S.CHAIN_MAXW
                                           for p in (self.priv, self.scan))
        self._build(shapes)

    # ------------------------------------------------------------------ argument lists
    def _build(self, shapes):
        a, pr, sc, es, cr = self.actor, self.priv, self.scan, self.est, self.critic
        # 1. weight split jobs (after every Adam step)
        self.wsplit = []
        for p in self.parts:
            for l, W in enumerate(p.W):
                Ws = p.Ws[l]
                if p is a and l == 0:
                    for (c, s8, w) in self.spans:
                        if w:
                            self.wsplit.append(S.split_job(W.detach()[:, c:c + w], S.group_ptr(Ws, s8), Ws.shape[1]))
                else:
                    self.wsplit.append(S.split_job(W.detach(), Ws.data_ptr(), Ws.shape[1]))
        # the chained encoders' weights also fragment-packed (the chain kernel's B loads)
        # (forward), and their transposes (input gradients of the layers past the first)
        for p in ((pr, sc) if self.enc_chain else ()):
            p.Wp = [S.packed_empty(W.shape[0], W.shape[1], self.dev) for W in p.W]
            for W, Wp in zip(p.W, p.Wp):
                self.wsplit.append(S.split_packed_job(W.detach(), Wp))
        self._fwd_levels = None  # built per minibatch offset (input row pointers)
        self._shapes = shapes
        # the same S8 destinations as optimizer-tail entries (lgx_tail_s8_seg): the Adam launch
        # writes each updated weight's S8 copies itself, so only an update's first minibatch needs
        # the split launch (prepare); None where a weight is not a view of the flat parameters
        self.tail_segs = self._tail_segments()
        self._tail_dev = None

    def _tail_segments(self):
        """[(p0, N, K, c0, w, dst, ld, packed)] of every S8 weight copy (include/lgx_mlp.h
        lgx_tail_s8_seg), or None."""
        pb = getattr(self.alg, "params_buf", None)
        if pb is None or not H.TAIL_S8 or pb.dtype != torch.float32:
            return None
        base, end = pb.data_ptr(), pb.data_ptr() + 4 * pb.numel()
        segs = []
        for p in self.parts:
            for l, W in enumerate(p.W):
                a = W.data_ptr()
                if not (base <= a < end) or (a - base) % 4 or not W.is_contiguous():
                    return None
                N, K = W.shape
                Ws = p.Ws[l]
                if p is self.actor and l == 0:
                    for (c, s8, w) in self.spans:
                        if w:
                            segs.append(((a - base) // 4, N, K, c, w, S.group_ptr(Ws, s8), Ws.shape[1], 0))
                else:
                    segs.append(((a - base) // 4, N, K, 0, K, Ws.data_ptr(), Ws.shape[1], 0))
        for p in ((self.priv, self.scan) if self.enc_chain else ()):
            for W, Wp in zip(p.W, p.Wp):
                N, K = W.shape
                segs.append(((W.data_ptr() - base) // 4, N, K, 0, K, Wp.data_ptr(), (K + 31) // 32, 1))
        return segs if len(segs) <= H.TAIL_S8_MAX else None

    def tail_table(self):
        """(host table, count) for lgx_ppo_tail, or None (the split then runs per minibatch)."""
        if self.tail_segs is None:
            return None
        if self._tail_dev is None:
            self._tail_dev = H.tail_s8_table(self.tail_segs)
        return self._tail_dev, len(self.tail_segs)

    def _fwd(self, p, l, A_ptr, lda, K, C=None, ldc=0, C32=None, ldc32=0, elu=True, n0=0, n1=None):
        """Layer l's forward GemmArgs; n0, n1: only output columns [n0, n1) (C already offset)."""
        W = p.W[l]
        Ws = p.Ws[l]
        n1 = W.shape[0] if n1 is None else n1
        return S.GemmArgs(A=A_ptr, lda=lda, B=Ws.data_ptr() + 4 * n0 * Ws.shape[1], ldb=Ws.shape[1], M=self.mb,
                          N=n1 - n0, K=K, epilogue=S.EPI_BIAS | (S.EPI_ELU if elu else 0), C=C, ldc=ldc, C32=C32,
                          ldc32=ldc32, bias=p.b[l].data_ptr() + 4 * n0)

    @staticmethod
    def _slices(N, ns):
        """ns column ranges of [0, N), boundaries at multiples of 8 (S8 groups)."""
        b = [min(N, (N * q // ns + 7) // 8 * 8) for q in range(ns)] + [N]
        return [(b[q], b[q + 1]) for q in range(ns) if b[q] < b[q + 1]]

    def prepare(self, perm, flat):
        """Per update: the network inputs of every row, permuted, into S8 (one launch).
        flat: storage._flat() (obs, priv, critic, est, scan, ...)."""
        obs, priv, critic, est, scan = flat[:5]
        jobs = [S.split_job(obs, self.ain.data_ptr(), self.ain.shape[1], idx=perm, rows=self.rows),
                S.split_job(est, S.group_ptr(self.ain, self.P2), self.ain.shape[1], idx=perm, rows=self.rows),
                S.split_job(critic, self.crin.data_ptr(), self.crin.shape[1], idx=perm, rows=self.rows),
                S.split_job(priv, self.prin.data_ptr(), self.prin.shape[1], idx=perm, rows=self.rows),
                S.split_job(scan, self.scin.data_ptr(), self.scin.shape[1], idx=perm, rows=self.rows)]
        # with tail_segs the update's weights too (the optimizer tail keeps the copies current)
        S.split(jobs + (self.wsplit if self.tail_segs is not None else []))

    # ------------------------------------------------------------------ one minibatch
    def run(self, i, shuf, adapt_latent, head_out, aux_out, kl_dst):
        """Minibatch i (rows [i mb, (i + 1) mb) of the permuted inputs): forward, loss heads,
        backward, gradients into the flat buffer (alg.grads), loss values into head_out/aux_out."""
        alg = self.alg
        mb = self.mb
        r0 = i * mb
        a, pr, sc, es, cr = self.actor, self.priv, self.scan, self.est, self.critic
        row = lambda buf, col=0: S.group_ptr(buf, col) + 4 * r0 * buf.shape[1]  # noqa: E731
        lda_ain = self.ain.shape[1]
        # 1. weights -> S8 (with tail_segs: once per update in prepare, then by the optimizer tail)
        if self.tail_segs is None:
            S.split(self.wsplit)
        # 2. forward
        ins = {"priv": (row(self.prin), self.prin.shape[1], pr.W[0].shape[1]),
               "scan": (row(self.scin), self.scin.shape[1], sc.W[0].shape[1]),
               "est": (row(self.ain, self.est_c0), lda_ain, self.est_k),
               "critic": (row(self.crin), self.crin.shape[1], cr.W[0].shape[1])}
        enc_depth = max(pr.n, sc.n)
        levels = {}

        def put(level, args):
            levels.setdefault(level, []).append(args)
        chains = []
        for p in (pr, sc, es, cr):
            A_ptr, lda, K = ins[p.name]
            if self.enc_chain and p in (pr, sc):
                c = S.ChainArgs(A=A_ptr, lda=lda, rows=mb, nlayers=p.n)
                for l in range(p.n):
                    W = p.W[l]
                    L = c.layers[l]
                    L.W, L.packed, L.bias = p.Wp[l].data_ptr(), 1, p.b[l].data_ptr()
                    L.K, L.N, L.elu = W.shape[1], W.shape[0], int(l < p.n - 1)
                    if l < p.n - 1:
                        L.C, L.ldc = p.out[l].data_ptr(), p.out[l].shape[1]
                    elif p is pr:
                        L.C, L.ldc, L.C32, L.ldc32 = row(self.ain, self.P0), lda_ain, self.lat.data_ptr(), self.nlat
                    else:
                        L.C, L.ldc = row(self.ain, self.P1), lda_ain
                chains.append(c)
                continue
            sh = self.fwd_shift.get(p.name, 0)
            for l in range(p.n):
                last = l == p.n - 1
                if not last:
                    o = p.out[l]
                    ns = self.l0_slices.get(p.name, 1) if l == 0 else 1
                    if ns > 1:
                        # column slices of a first layer in the levels before its own (the
                        # privileged / scan encoders' narrow levels), the last slice at l + sh
                        for q, (n0, n1) in enumerate(self._slices(p.W[0].shape[0], ns)):
                            put(l + sh - (ns - 1) + q, self._fwd(p, l, A_ptr, lda, K, C=S.group_ptr(o, n0),
                                                                 ldc=o.shape[1], n0=n0, n1=n1))
                    else:
                        put(l + sh, self._fwd(p, l, A_ptr, lda, K, C=o.data_ptr(), ldc=o.shape[1]))
                    A_ptr, lda, K = o.data_ptr(), o.shape[1], p.W[l].shape[0]
                    continue
                if p is pr:
                    put(l, self._fwd(p, l, A_ptr, lda, K, C=row(self.ain, self.P0), ldc=lda_ain,
                                     C32=self.lat.data_ptr(), ldc32=self.nlat, elu=False))
                elif p is sc:
                    put(l, self._fwd(p, l, A_ptr, lda, K, C=row(self.ain, self.P1), ldc=lda_ain, elu=False))
                elif p is es:
                    put(l + sh, self._fwd(p, l, A_ptr, lda, K, C32=self.pred.data_ptr(), ldc32=self.pred.shape[1],
                                          elu=False))
                elif not self.tail:
                    put(l + sh, self._fwd(p, l, A_ptr, lda, K, C32=self.value.data_ptr(), ldc32=1, elu=False))
        A_ptr, lda, K = row(self.ain), lda_ain, self.W8
        for l in range(a.n):
            lev = enc_depth + l
            if l < a.n - 1:
                o = a.out[l]
                put(lev, self._fwd(a, l, A_ptr, lda, K, C=o.data_ptr(), ldc=o.shape[1]))
                A_ptr, lda, K = o.data_ptr(), o.shape[1], a.W[l].shape[0]
            elif not self.tail:
                put(lev, self._fwd(a, l, A_ptr, lda, K, C32=self.mu.data_ptr(), ldc32=self.mu.shape[1], elu=False))
        if chains:
            S.chain(chains)
        for lev in sorted(levels):
            S.gemm_group(levels[lev], S.FWD)
        # 3. loss heads: forward sums and input gradients in one launch; the narrow output
        #    gradients straight into S8 with their per-256-row column sums (the last layers'
        #    bias gradients)
        (obs_b, priv_b, critic_b, est_b, scan_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b, old_mu_b,
         old_sigma_b) = shuf
        A = self.mu.shape[1]
        std = alg.actor_critic.std
        cnt, cnt_aux = H._counter(self.dev), H._counter(self.dev, "aux")
        seeds = alg._seeds  # [1, c_value, -c_entropy, c_reg, 1]
        h = H.HeadArgs(mu=self.mu.data_ptr(), value=self.value.data_ptr(), std=std.data_ptr(),
                       actions=actions_b.data_ptr(), old_logp=old_logp_b.data_ptr(), adv=adv_b.data_ptr(),
                       target_values=target_values_b.data_ptr(), returns=returns_b.data_ptr(),
                       old_mu=old_mu_b.data_ptr(), old_sigma=old_sigma_b.data_ptr(), B=mb, A=A,
                       clip=float(alg.clip_param), clipped_value=int(bool(alg.use_clipped_value_loss)),
                       out=head_out.data_ptr(), g=seeds.data_ptr(), dstd=std.grad.data_ptr(),
                       ws=self.head_ws.data_ptr(), counter=cnt.data_ptr(),
                       kl_dst=None if kl_dst is None else kl_dst.data_ptr(), accumulate_dstd=0)
        x = H.AuxArgs(p=self.lat.data_ptr(), a=adapt_latent.data_ptr(), L=self.nlat, e=self.pred.data_ptr(),
                      t=est_b.data_ptr(), E=self.pred.shape[1], B=mb, out=aux_out.data_ptr(), g=seeds.data_ptr() + 12,
                      dp=self.dp.data_ptr(), ws=self.aux_ws.data_ptr(), counter=cnt_aux.data_ptr(), ld_p=self.nlat)
        s8 = H.HeadsS8Args(dmu_s8=a.dy[-1].data_ptr(), ld_dmu=a.dy[-1].shape[1], dmu_cs=a.cs[-1].data_ptr(),
                           dvalue_s8=cr.dy[-1].data_ptr(), ld_dvalue=cr.dy[-1].shape[1], dvalue_cs=cr.cs[-1].data_ptr(),
                           de_s8=es.dy[-1].data_ptr(), ld_de=es.dy[-1].shape[1], de_cs=es.cs[-1].data_ptr())
        dec = getattr(alg, "_decisions", None)
        if dec is not None:
            # test hook (tests/learner_replay.py, eager updates only): the k-th minibatch's
            # per-sample clip / max decisions replayed from a reference run ("in") and / or
            # recorded ("out"), include/lgx_mlp.h lgx_heads_s8_args
            k = dec["k"]
            dec["k"] = k + 1
            s8.decisions_in = dec["in"][k].data_ptr() if dec.get("in") is not None else None
            s8.decisions_out = dec["out"][k].data_ptr() if dec.get("out") is not None else None
        if self.tail:
            t = H.HeadsTailArgs(y=a.out[-1].data_ptr(), ld_y=a.out[-1].shape[1], W=a.W[-1].data_ptr(),
                                b=a.b[-1].data_ptr(), dy=a.dy[-2].data_ptr(), ld_dy=a.dy[-2].shape[1],
                                dy_cs=a.cs[-2].data_ptr(), yc=cr.out[-1].data_ptr(), ld_yc=cr.out[-1].shape[1],
                                Wc=cr.W[-1].data_ptr(), bc=cr.b[-1].data_ptr(), dyc=cr.dy[-2].data_ptr(),
                                ld_dyc=cr.dy[-2].shape[1], dyc_cs=cr.cs[-2].data_ptr(), mu_out=self.mu.data_ptr(),
                                value_out=self.value.data_ptr(), H=a.W[-1].shape[1], Hc=cr.W[-1].shape[1])
            H._check(H.lib().lgx_loss_heads_tail(H.C.byref(h), H.C.byref(x), H.C.byref(s8), H.C.byref(t),
                                                 H._stream()), "lgx_loss_heads_tail")
        else:
            H._check(H.lib().lgx_loss_heads_fused(H.C.byref(h), H.C.byref(x), H.C.byref(s8), H._stream()),
                     "lgx_loss_heads_fused")
        # 4. input gradients
        blev = {}

        def bput(level, args):
            blev.setdefault(level, []).append(args)

        def dx(p, l, dy, dst, cs, N=None, Bptr=None, elu=True, addend=None):
            W = p.W[l]
            Ws = p.Ws[l]
            return S.GemmArgs(A=dy.data_ptr(), lda=dy.shape[1], B=Ws.data_ptr() if Bptr is None else Bptr,
                              ldb=Ws.shape[1], M=mb, N=W.shape[1] if N is None else N, K=W.shape[0],
                              epilogue=S.EPI_DELU if elu else 0, C=dst if isinstance(dst, int) else dst.data_ptr(),
                              ldc=self.dlat.shape[1] if isinstance(dst, int) else dst.shape[1],
                              act=None if not elu else p.out[l - 1].data_ptr(),
                              ld_act=0 if not elu else p.out[l - 1].shape[1],
                              addend=None if addend is None else addend.data_ptr(),
                              ld_add=0 if addend is None else addend.stride(0),
                              add_cols=0 if addend is None else addend.shape[1], colsum_ws=cs.data_ptr())
        for p in (a, cr, es):
            sh = self.dx_shift.get(p.name, 0)
            for l in range(p.n - 1, 0, -1):
                if self.tail and p is not es and l == p.n - 1:
                    continue  # in the heads-tail launch
                bput(p.n - 1 - l + sh, dx(p, l, p.dy[l], p.dy[l - 1], p.cs[l - 1]))
        # the actor's first layer: gradient of its latent columns (+ the regulariser's)
        lev_lat = a.n - 1
        bput(lev_lat, dx(a, 0, a.dy[0], self.dlat.data_ptr(), self.cs_lat, N=self.P2 - self.P0,
                         Bptr=S.group_ptr(a.Ws[0], self.P0), elu=False, addend=self.dp))
        for p, c0 in ((pr, 0), (sc, self.P1 - self.P0)):
            for l in range(p.n - 1, 0, -1):
                dy = self.dlat if l == p.n - 1 else p.dy[l]
                if l == p.n - 1:
                    args = S.GemmArgs(A=S.group_ptr(self.dlat, c0), lda=self.dlat.shape[1], B=p.Ws[l].data_ptr(),
                                      ldb=p.Ws[l].shape[1], M=mb, N=p.W[l].shape[1], K=p.W[l].shape[0],
                                      epilogue=S.EPI_DELU, C=p.dy[l - 1].data_ptr(), ldc=p.dy[l - 1].shape[1],
                                      act=p.out[l - 1].data_ptr(), ld_act=p.out[l - 1].shape[1],
                                      colsum_ws=p.cs[l - 1].data_ptr())
                else:
                    args = dx(p, l, dy, p.dy[l - 1], p.cs[l - 1])
                bput(lev_lat + 1 + (p.n - 1 - l), args)
        for lev in sorted(blev):
            S.gemm_group(blev[lev], S.DX)
        # 5. weight gradients (one launch) and the reductions into the flat gradient buffer
        g_args, red = [], []
        off = 0
        k = 0
        for p in self.parts:
            for l, W in enumerate(p.W):
                M, N, _K = self._shapes[k]
                s = self.splits[k]
                k += 1
                # A = dy[l] (TR), B = the layer input (TR)
                if p in (pr, sc) and l == p.n - 1:
                    dyp, ldy = S.group_ptr(self.dlat, 0 if p is pr else self.P1 - self.P0), self.dlat.shape[1]
                else:
                    dyp, ldy = p.dy[l].data_ptr(), p.dy[l].shape[1]
                if l > 0:
                    xp, ldx = p.out[l - 1].data_ptr(), p.out[l - 1].shape[1]
                else:
                    xp, ldx, _k = ins[p.name] if p is not a else (row(self.ain), lda_ain, self.W8)
                ws = self.dw_ws.data_ptr() + 4 * off
                g_args.append(S.GemmArgs(A=dyp, lda=ldy, B=xp, ldb=ldx, M=M, N=N, K=mb, C32=ws, ldc32=N, split=s))
                Wg = W.grad
                if p is a and l == 0:
                    for (c, s8, w) in self.spans:
                        if w:
                            red.append(S.ReduceArgs(ws=ws + 4 * s8, stride=M * N, ld_ws=N, out=Wg.data_ptr() + 4 * c,
                                                    ld_out=Wg.shape[1], rows=M, cols=w, nsplit=s, accumulate=0))
                else:
                    red.append(S.flat_reduce(ws, M * N, Wg.data_ptr(), M * N, s))
                off += s * M * N
        # bias gradients from the column-sum partials
        nsb, tm = self.nsb, self.tiles_m
        for p in self.parts:
            for l in range(p.n):
                bg = p.b[l].grad
                n = bg.numel()
                if p in (pr, sc) and l == p.n - 1:
                    c0 = 0 if p is pr else self.P1 - self.P0
                    # the tile partials of the latent columns: [tiles][P2 - P0]
                    red.append(S.flat_reduce(self.cs_lat.data_ptr() + 4 * c0, self.cs_lat.shape[1], bg.data_ptr(), n,
                                             tm))
                    continue
                from_split = l == p.n - 1  # the loss heads' gradients: lgx_s8_split partials (256 rows)
                if self.tail and p in (a, cr) and l >= p.n - 2:
                    cnt = self.ntail  # the heads-tail launch's 32-row partials
                else:
                    cnt = nsb if from_split else tm
                red.append(S.flat_reduce(p.cs[l].data_ptr(), n, bg.data_ptr(), n, cnt))
        if self.tail:
            # the PPO head's totals from its per-block rows (lgx_loss_heads_tail): the surrogate and
            # value losses, the KL (its output slot and the all-reduced KL slot), dstd
            ws, nt, A = self.head_ws.data_ptr(), self.ntail, self.mu.shape[1]
            red.append(S.flat_reduce(ws, 19, head_out.data_ptr(), 2, nt))
            red.append(S.flat_reduce(ws + 8, 19, head_out.data_ptr() + 12, 1, nt))
            if kl_dst is not None:
                red.append(S.flat_reduce(ws + 8, 19, kl_dst.data_ptr(), 1, nt))
            red.append(S.flat_reduce(ws + 12, 19, alg.actor_critic.std.grad.data_ptr(), A, nt))
        S.gemm_group(g_args, S.DW)
        S.reduce(red)
