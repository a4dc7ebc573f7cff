"""PPO.act's networks in ONE launch (include/lgx_s8.h lgx_s8_act; reference ppo.py:129-153,
actor_critic.py:79-115 / 190-226, support_networks.py:25-80).

The rollout step's estimator, scan encoder, privileged encoder, actor and critic run as one
kernel over S8 copies of their weights (bf16 hi / lo, packed as MFMA fragments: lgx_s8_act_pack):
32 envs per block, the activations in LDS, the actor input assembled in place as [obs | priv latent | scan
latent | est] in the update's segmented layout. The weights are packed once per rollout (at its
first step, inside the rollout graph). The kernel also writes this step's observation rows of
the storage (rollout_storage.py:87-105; no separate copy launch) and, given `head`, runs the act
head in the actor blocks (a = mu + std * eps, the Normal log-prob, the action / mu / sigma rows:
lgx_act_head's arithmetic, ppo.py:141-147), mu never leaving LDS. Adaptation-mode rollouts (the DAgger
iterations) run the same kernel with the latent from the adaptation encoder (one fused launch).

Numerics: the same 3 x bf16 products as the grouped launches; the actor's first layer sums its
input in the segmented order (the gaps are zeros), so mu differs from the grouped path by fp32
rounding only (tests/test_gpu_s8_act.py: within 1e-5)."""
import torch

from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H
from legged_gym_custom_amd.rsl_rl.modules import hip_s8 as S
from .s8_update import _chain


def _r8(x):
    return (x + 7) // 8 * 8


class S8Act:
    @staticmethod
    def supported(alg):
        if not alg.on_gpu:
            return False
        S.lib()  # a broken build raises (LGX_FUSED_ACT on): no silent fallback to the grouped launches
        ac, est = alg.actor_critic, alg.estimator
        chains = [_chain(ac.actor), _chain(ac.critic), _chain(ac.privileged_encoder_.priv_encoder),
                  _chain(ac.scan_encoder.scan_encoder), _chain(est.estimator)]
        if any(c is None or len(c) > S.ACT_MAXL for c in chains):
            return False
        if ac.num_scan_obs <= 0 or ac.num_privileged_obs <= 0:
            return False
        actor, critic, priv, scan, estc = chains
        nobs = ac.num_proprio * (1 + ac.history_buffer_length)
        nlat, nscan, nest = priv[-1].out_features, scan[-1].out_features, ac.num_estimated_obs
        width = (_r8(nobs) + _r8(nlat) + _r8(nscan) + _r8(nest) + 31) // 32 * 32
        if width > S.ACT_MAXIN or actor[0].in_features != nobs + nlat + nscan + nest:
            return False
        if any(m.out_features > S.ACT_MAXH for m in actor[:-1] + critic[:-1]):
            return False
        if any(m.out_features > S.ACT_MAXENC for c in (priv, scan, estc) for m in c[:-1]):
            return False
        c0 = 0 if est.use_history else nobs - ac.num_proprio
        return (c0 % 4 == 0 and critic[-1].out_features == 1 and critic[0].in_features % 32 == 0
                and scan[0].in_features <= S.ACT_MAXENC and priv[0].in_features <= S.ACT_MAXENC)

    def __init__(self, alg, num_envs):
        """The estimator and the scan / privileged encoders run as grouped launches before the
        kernel (inside it, the actor blocks' 13 dependent layers measured slower)."""
        ac, est = alg.actor_critic, alg.estimator
        self.alg = alg
        dev = alg.device
        self.B = num_envs
        actor, critic = _chain(ac.actor), _chain(ac.critic)
        priv, scan = _chain(ac.privileged_encoder_.priv_encoder), _chain(ac.scan_encoder.scan_encoder)
        estc = _chain(est.estimator)
        nobs = ac.num_proprio * (1 + ac.history_buffer_length)
        nlat, nscan, nest = priv[-1].out_features, scan[-1].out_features, ac.num_estimated_obs
        P0 = _r8(nobs)
        P1 = P0 + _r8(nlat)
        P2 = P1 + _r8(nscan)
        width = (P2 + _r8(nest) + 31) // 32 * 32
        spans = [(0, 0, nobs), (nobs, P0, nlat), (nobs + nlat, P1, nscan), (nobs + nlat + nscan, P2, nest)]
        self.nobs, self.width = nobs, width
        self.est_c0 = 0 if est.use_history else nobs - ac.num_proprio
        self._keep = []  # packed weight buffers (their addresses are in the argument block)
        self.wpack = []
        a = S.ActArgs()
        a.B, a.width = num_envs, width
        a.seg[0], a.seg[1], a.seg[2], a.seg[3] = 0, P0, P1, P2
        a.est_c0 = self.est_c0

        def fill(dst, layers, first_actor=False):
            for i, m in enumerate(layers):
                W = m.weight.detach()
                N, K = W.shape
                sp = spans if first_actor and i == 0 else [(0, 0, K)]
                if first_actor and i == 0:
                    K = width
                steps = (K + 31) // 32
                Wp = torch.zeros(((N + 15) // 16) * steps * 2048 // 4, dtype=torch.int32, device=dev)
                j = S.ActPackArgs(W=W.data_ptr(), ld=W.stride(0), dst=Wp.data_ptr(), N=N, steps=steps, nspans=len(sp))
                for q, (c, p0, w) in enumerate(sp):
                    j.span_c0[q], j.span_p0[q], j.span_w[q] = c, p0, w
                self.wpack.append(j)
                self._keep.append(Wp)
                dst[i] = S.ActLayer(W=Wp.data_ptr(), ldw=steps, b=m.bias.data_ptr(), K=K, N=N,
                                    elu=int(i < len(layers) - 1))
            return len(layers)
        # the encoders' outputs: spans of one [B, latent | scan latent | est] buffer
        self.parts = torch.empty(num_envs, nlat + nscan + nest, device=dev)
        self.spans = [self.parts[:, :nlat], self.parts[:, nlat:nlat + nscan], self.parts[:, nlat + nscan:]]
        for q, t in enumerate(self.spans):
            a.part_src[q], a.part_ld[q], a.part_w[q] = t.data_ptr(), t.stride(0), t.shape[1]
        a.n_actor = fill(a.actor, actor, first_actor=True)
        a.n_critic = fill(a.critic, critic)
        self.mu = torch.empty(num_envs, actor[-1].out_features, device=dev)
        self.value = torch.empty(num_envs, 1, device=dev)
        a.mu, a.ld_mu, a.value = self.mu.data_ptr(), self.mu.stride(0), self.value.data_ptr()
        self.args = a

    def refresh_weights(self):
        """The weights -> the kernel's packed S8 fragments (one launch; the rollout's first step,
        after the update changed them)."""
        S.act_pack(self.wpack)

    def run(self, obs, priv, critic, scan, est=None, rows=None, head=None, adaptation_mode=False):
        """(mu [B, A], value [B, 1]) of this step's observations (static output buffers).
        rows (optional): this step's storage rows [obs, priv, critic, est, scan] (contiguous),
        which the kernel fills from the inputs (est: the true estimated obs, copied only).
        head (optional): dict(std, eps, actions, mu, sigma, logp, actions_copy, noise) as
        hip_mlp.act_head takes them; the kernel then writes those rows and NOT the mu buffer
        (mu is returned as None). adaptation_mode: the actor's latent from the adaptation encoder
        over the observation history (the DAgger iterations' rollout, actor_critic.py:75-76, one
        lgx_adaptation_forward launch into the latent span) instead of the privileged encoder."""
        a = self.args
        if head is None:
            a.actions = None
        else:
            A = self.mu.shape[1]
            outs = [head[k] for k in ("actions", "mu", "sigma", "logp")]
            cp = head.get("actions_copy")
            for t in outs[:3] + ([cp] if cp is not None else []):
                if t.shape != (self.B, A) or not t.is_contiguous() or t.dtype != torch.float32:
                    raise S.S8LibError("S8Act: act-head rows must be contiguous fp32 [num_envs, A]")
            if outs[3].numel() != self.B or not outs[3].is_contiguous():
                raise S.S8LibError("S8Act: log-prob row must be contiguous [num_envs]")
            eps = head.get("eps")
            if eps is None:
                seed, step_dev, off = head["noise"]
                if step_dev.dtype != torch.int64 or step_dev.device != self.mu.device:
                    raise S.S8LibError("S8Act: step_dev must be an int64 tensor on the device")
                a.eps, a.step_dev, a.seed, a.env_offset = None, step_dev.data_ptr(), int(seed) & (2**64 - 1), int(off)
            else:
                if eps.shape != (self.B, A) or not eps.is_contiguous():
                    raise S.S8LibError("S8Act: eps must be contiguous [num_envs, A]")
                a.eps, a.step_dev, a.seed, a.env_offset = eps.data_ptr(), None, 0, 0
            a.std = head["std"].data_ptr()
            a.actions, a.mu_st, a.sigma_st, a.logp_st = (t.data_ptr() for t in outs)
            a.actions_copy = None if cp is None else cp.data_ptr()
            self._head_keep = head  # the argument block holds their addresses
        for t in (obs, priv, critic, scan) + (() if est is None else (est,)):
            if t.stride(1) != 1 or t.dtype != torch.float32 or t.shape[0] != self.B:
                raise S.S8LibError("S8Act: fp32 [num_envs, cols] inputs with unit column stride")
        a.obs, a.ld_obs, a.n_obs = obs.data_ptr(), obs.stride(0), obs.shape[1]
        a.priv_obs, a.ld_priv, a.n_priv_in = priv.data_ptr(), priv.stride(0), priv.shape[1]
        a.critic_obs, a.ld_critic, a.n_critic_in = critic.data_ptr(), critic.stride(0), critic.shape[1]
        a.scan_obs, a.ld_scan, a.n_scan_in = scan.data_ptr(), scan.stride(0), scan.shape[1]
        if rows is not None:
            src = (obs, priv, critic, est, scan)
            for d, x in zip(rows, src):
                if not d.is_contiguous() or d.shape != x.shape:
                    raise S.S8LibError("S8Act: storage rows must be contiguous and shaped as the inputs")
            a.obs_st, a.priv_st, a.critic_st, a.est_st, a.scan_st = (d.data_ptr() for d in rows)
            a.est_obs, a.ld_est, a.n_est_obs = est.data_ptr(), est.stride(0), est.shape[1]
        else:
            a.obs_st = a.priv_st = a.critic_st = a.est_st = a.scan_st = a.est_obs = None
        a.nets = 0
        # the estimator and the scan / privileged encoders: grouped launches writing their
        # outputs into the spans the kernel reads
        alg = self.alg
        ac = alg.actor_critic
        e_mod, e_in = alg.estimator.group_item(obs)
        s_mod, s_in = ac.scan_encoder.group_item(scan)
        items = [(e_mod, e_in, None, self.spans[2]), (s_mod, s_in, None, self.spans[1])]
        if not adaptation_mode:
            p_mod, p_in = ac.privileged_encoder_.group_item(priv)
            items.append((p_mod, p_in, None, self.spans[0]))
        H.forward_group(items)
        if adaptation_mode:
            P = ac.num_proprio
            hist = obs[:, :obs.shape[1] - P].reshape(self.B, ac.history_buffer_length, P)
            H.adaptation_forward_into(ac.adaptation_encoder_, hist, self.spans[0])
        S.act(a)
        return (self.mu if head is None else None), self.value
