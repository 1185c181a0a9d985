"""Native engine for the reference's MLP actor-critic (kernels K01/K02/K05/K07/K08 of SURVEY §2.4, ``mlp.hip``).

The reference builds its actor and critic as separate TF graphs (``Basic_AC/policies.py:33-162``,
``A3C/policies.py:34-182``) and runs each ``Session.run`` as ~10 TF ops per layer. Here each tower is ONE workgroup
per 16 rows with its activations in LDS, on f32 MFMA:

* :meth:`MLPEngine.policy_step` -- rollout: both towers in one launch; the actor workgroups also sample the action
  (Gaussian Box-Muller / categorical Gumbel-max, counter-based keys derived from the env counters, so the actions are
  bit-identical to :func:`..ops.distributions.gaussian_sample_ref` draws), and write log-prob and entropy; the critic
  workgroups write V(s).
* :meth:`MLPEngine.train` -- learner (mini)batch: one fused launch (gathered rows -> forward -> per-row loss gradient
  -> data-gradient chain) + one weight-gradient launch (every dW/db element written once, deterministic; per-tile
  sums of squares for the global-norm clip; loss statistics). The optimiser step follows (:mod:`.optim`).
* :meth:`MLPEngine.evaluate` / :meth:`value` -- log-prob / entropy of given actions and values (post-update KL proxy
  and EV of the reference, ``Basic_AC/run_AC.py:257-258``; bootstrap values).
* :meth:`MLPEngine.rollout_linear` -- the whole T-step rollout of the MuJoCo-shaped bank in ONE persistent launch
  (actor on 4x4x1 MFMA tiles + sampling + env dynamics + frame stack per 4-env workgroup, ``mlp_rollout_kernel``) followed by ONE
  batched critic launch over all ``(T+1) N`` observations (the rollout's Session.run-per-step loop of
  ``Basic_AC/run_AC.py:82-107``).

Weights are read in place from the fp32 parameter slab (TF ``[in, out]`` kernels, so checkpoints need no
transposes) and gradients are written straight into the gradient slab.
"""
from __future__ import annotations

import torch

from .. import _native

MAXL = 5
TOWER_WORDS = 2 + 11 * MAXL    # int64 words of one MlpTower (csrc/kernels/mlp_desc.h)
ACT_CODES = {None: 0, "none": 0, "relu": 1, "lrelu": 2, "tanh": 3}
BM = 16
MAXW = 256
PARTS = 256
MPART_W = 24    # per-workgroup partial row of the train kernel (mlp_desc.h)
LIN_OBS, LIN_ACT = 17, 6


def ngp2(w):
    """16-wide groups of a width rounded up to a power of two (common.h mlp_ngp2)."""
    g = (w + 15) // 16
    return 1 if g <= 1 else 2 if g <= 2 else 4 if g <= 4 else 8 if g <= 8 else 16


def _ld(w):
    """LDS row stride of a width (mlp.hip ld_of: 16 * power-of-two k-groups + 4)."""
    return 16 * ngp2(w) + 4


def _nct(w):
    """16-wide column tiles of a width (the training workspace's blocks per row tile)."""
    return (w + 15) // 16


def frag_f(W):
    """Forward fragment copy of a [K][N] weight (common.h mlp_frag_f): [ngp2(N) tiles][ngp2(K) groups][64 lanes][4],
    zero pad -- the layout the optimiser step and ``mlp_tshadow`` write."""
    K, N = W.shape
    gk, tn = ngp2(K), ngp2(N)
    P = torch.zeros(16 * gk, 16 * tn, dtype=W.dtype, device=W.device)
    P[:K, :N] = W
    # (tile, r) = c, (g, q, s) = k: element at ((tile * gk + g) * 64 + q * 16 + r) * 4 + s
    return P.reshape(gk, 4, 4, tn, 16).permute(3, 0, 1, 4, 2).reshape(-1)


def frag_g(W):
    """Data-gradient fragment copy of a [K][N] weight (common.h mlp_frag_g): [ngp2(K) tiles][ngp2(N) groups][64][4]."""
    return frag_f(W.t())


class MLPEngine:
    def __init__(self, model, flat):
        from ..models.policy import MLPActorCritic
        assert isinstance(model, MLPActorCritic)
        self.model = model
        self.flat = flat
        self.dev = flat.data.device
        actor, critic = model.actor, model.critic
        self.discrete = model.discrete
        self.D = actor.ob_dim
        self.A = actor.ac_dim
        self.head = 1 if self.discrete else 2
        if self.A > 16:
            raise ValueError("MLP engine heads support at most 16 actions")
        out_layer = actor.logits if self.discrete else actor.mu_layer
        self.towers = [
            [actor.first_layer, actor.second_layer, actor.third_layer, out_layer],
            [critic.first_layer, critic.second_layer] + ([critic.third_layer] if critic.variant == "a3c" else [])
            + [critic.value],
        ]
        for tw in self.towers:
            assert len(tw) <= MAXL and tw[0].in_features == self.D
            for i, lay in enumerate(tw):
                assert lay.in_features <= MAXW and lay.out_features <= MAXW
                # layer widths above 32 must be multiples of 16 (vectorised data-gradient weight loads, mlp.hip)
                assert lay.out_features <= 32 or lay.out_features % 16 == 0
                if i:
                    assert lay.in_features == tw[i - 1].out_features
        idx = {id(p): i for i, p in enumerate(flat.params)}

        def views(p):
            i = idx[id(p)]
            off, n = flat.offsets[i], p.numel()
            return flat.data[off:off + n], flat.grad[off:off + n]

        self._views = views
        if not self.discrete:
            self.log_std, self.g_log_std = views(actor.log_std)
            self.ac_scale = actor.ac_scale.to(self.dev, torch.float32).contiguous()
        else:
            self.log_std = self.g_log_std = self.ac_scale = None
        self.mstats = torch.zeros(8, dtype=torch.float32, device=self.dev)
        self.parts = [torch.zeros(PARTS, dtype=torch.float32, device=self.dev) for _ in range(2)]
        self.items = [sum(((l.in_features + 15) // 16) * ((l.out_features + 15) // 16) for l in tw)
                      for tw in self.towers]
        self._descs = {}
        self._hdescs = {}
        self._witems = {}
        self._mparts = {}
        self._dummy_stats = torch.zeros(16, dtype=torch.float32, device=self.dev)
        # fp32 FRAGMENT copies of every weight (common.h mlp_frag_f / mlp_frag_g, zero pad): F, the forward's B
        # operand, for every layer; G, the data gradient's, for layers >= 1 (layer 0 has no data gradient)
        self.F, self.G = {}, {}
        for tw in self.towers:
            for i, lay in enumerate(tw):
                n = ngp2(lay.in_features) * ngp2(lay.out_features) * 256
                self.F[id(lay)] = torch.zeros(n, dtype=torch.float32, device=self.dev)
                if i:
                    self.G[id(lay)] = torch.zeros(n, dtype=torch.float32, device=self.dev)
        self.n_weights = sum(l.in_features * l.out_features for tw in self.towers for l in tw)
        # reference tower shapes: the train launches take the SPEC path (every weight fragment preloaded, mlp.hip)
        self.spec = True
        self.sync_shadow()

    def frag_copies(self):
        """Per tower (= optimiser group actor, critic): (W view, K, N, F, G or None) -- the fragment copies the
        optimiser step writes as it goes (``ops/optim.py`` FusedGroupStep item tables)."""
        return [[(self._views(l.kernel)[0], l.in_features, l.out_features, self.F[id(l)], self.G.get(id(l)))
                 for l in tw] for tw in self.towers]

    def sync_shadow(self):
        """Rewrites the weight fragment copies from the fp32 slab (the optimiser step writes them itself; this pass
        covers engine creation and parameter changes outside it: checkpoint load, broadcast, parameter-server pull)."""
        desc, _ = self.desc(None)
        _native.require().mlp_tshadow(desc, 2, self.n_weights)

    # ------------------------------------------------------------------------------------------- descriptors
    def desc(self, B=None):
        """Device descriptor (+ training workspace for batch ``B``; ``None`` = inference only)."""
        if B in self._descs:
            return self._descs[B]
        words = torch.zeros(2 * TOWER_WORDS, dtype=torch.int64)
        ws = []
        for t, tw in enumerate(self.towers):
            base = t * TOWER_WORDS
            words[base] = len(tw)
            for l, lay in enumerate(tw):
                W, gW = self._views(lay.kernel)
                b, gb = self._views(lay.bias)
                words[base + 2 + l] = lay.in_features
                words[base + 2 + MAXL + l] = lay.out_features
                words[base + 2 + 2 * MAXL + l] = ACT_CODES[lay.activation]
                for j, tns in enumerate((W, b, gW, gb)):
                    words[base + 2 + (3 + j) * MAXL + l] = tns.data_ptr()
                words[base + 2 + 9 * MAXL + l] = self.F[id(lay)].data_ptr()
                if id(lay) in self.G:
                    words[base + 2 + 10 * MAXL + l] = self.G[id(lay)].data_ptr()
                if B is not None:
                    # 16 x 16 blocks, column-major inside (mlp.hip blk_out), one row of blocks per 16-row tile
                    nrt = (B + BM - 1) // BM
                    xs = torch.zeros(nrt * _nct(lay.in_features) * 256, dtype=torch.float32, device=self.dev)
                    dp = torch.zeros(nrt * _nct(lay.out_features) * 256, dtype=torch.float32, device=self.dev)
                    ws += [xs, dp]
                    words[base + 2 + 7 * MAXL + l] = xs.data_ptr()
                    words[base + 2 + 8 * MAXL + l] = dp.data_ptr()
        d = (words.to(self.dev), ws)
        self._descs[B] = d
        self._hdescs[B] = words   # CPU copy: the SPEC train path takes the tower descriptors as kernel arguments
        return d

    def lds_bytes(self, mode, tw_base, ntw):
        best = 0
        for t in range(tw_base, tw_base + ntw):
            n = BM * _ld(self.D)
            for lay in self.towers[t]:
                n += BM * _ld(lay.out_features)
            if mode == 2:
                n += 2 * BM * (MAXW + 4)
            best = max(best, n)
        return best * 4

    def _mpart(self, B):
        """Per-workgroup partial rows of the train kernel (loss statistics + log-std gradient), summed by the
        weight-gradient kernel -- no same-address atomics from every workgroup."""
        if B not in self._mparts:
            self._mparts[B] = torch.zeros((B + BM - 1) // BM * MPART_W, dtype=torch.float32, device=self.dev)
        return self._mparts[B]

    def _fwd(self, mode, obs, B, tw_base=0, ntw=2, desc_B=None, idx=None, perm=None, tg=None, env_ids=None, key_shift=0,
             seed=0, act_out=None, logp_out=None, ent_out=None, v_out=None, act_in=None, logp_old=None, adv=None,
             ret=None, v_old=None, ent_coef=None, kl_coef=None, vf_coef=1.0, ppo_clip=0.0, v_clip=0.0, ppo=False,
             stamps=None):
        ops = _native.require()
        desc, _ = self.desc(desc_B)
        obs2 = obs.reshape(obs.shape[0], -1)
        puc, pep, poff, pn, pseed = perm if perm is not None else (None, 0, 0, 0, 0)
        ops.mlp_fwd(desc, tw_base, ntw, mode, self.lds_bytes(mode, tw_base, ntw), obs2, idx, puc, pep, poff, pn,
                    pseed, B, self.head, self.A,
                    self.log_std, self.ac_scale, tg, env_ids, key_shift, seed, act_out, logp_out, ent_out, v_out,
                    act_in, logp_old, adv, ret, v_old, ent_coef, kl_coef, float(vf_coef), float(ppo_clip),
                    float(v_clip or 0.0), bool(ppo), self.g_log_std if mode == 2 else None,
                    self.mstats if mode == 2 else None, self._mpart(B) if mode == 2 else None, stamps,
                    self._hdescs[desc_B] if (mode == 2 and self.spec) else None)

    # ------------------------------------------------------------------------------------------- API
    def policy_step(self, obs, act_out, logp_out, ent_out, v_out, tg, env_ids, key_shift, seed):
        """Rollout step over the env bank: actions, log-probs, entropies and values in one launch."""
        self._fwd(0, obs, obs.shape[0], 0, 2, tg=tg, env_ids=env_ids, key_shift=key_shift, seed=seed,
                  act_out=act_out, logp_out=logp_out, ent_out=ent_out, v_out=v_out)

    def value(self, obs, out):
        self._fwd(1, obs, obs.shape[0], 1, 1, v_out=out)
        return out

    def evaluate(self, obs, actions, logp_out, ent_out=None, v_out=None):
        self._fwd(1, obs, obs.shape[0], 0, 2 if v_out is not None else 1, act_in=actions, logp_out=logp_out,
                  ent_out=ent_out, v_out=v_out)

    def train(self, obs, actions, logp_old, adv, ret, ent_coef, kl_coef, B, idx=None, v_old=None, vf_coef=1.0,
              ppo=False, ppo_clip=0.0, v_clip=0.0, stats=None, clips=(None, None), want_parts=True, perm=None,
              bump=None, stamps=None):
        """One learner (mini)batch: rows ``idx`` / ``perm`` = (update_counter, epoch, offset, n, seed) -- the rows
        ``prp(offset + r)`` of the keyed permutation of ``[0, n)`` (envs/rng.py), computed in-kernel -- or the first
        ``B`` rows of the rollout -> gradients in the slab, statistics into ``stats[0:7]``, sums of squares into
        :attr:`parts` (when ``want_parts``). ``bump``: an int64 counter the weight-gradient launch advances by one
        (the PPO update counter, after the update's last minibatch -- no separate launch)."""
        ops = _native.require()
        self._fwd(2, obs, B, 0, 2, desc_B=B, idx=idx, perm=perm, act_in=actions, logp_old=logp_old, adv=adv, ret=ret,
                  v_old=v_old, ent_coef=ent_coef, kl_coef=kl_coef, vf_coef=vf_coef, ppo_clip=ppo_clip,
                  v_clip=v_clip, ppo=ppo, stamps=stamps)
        nrt = (B + BM - 1) // BM
        nsplit = max(1, min(16, nrt // 128))
        self.last_stores_all = nsplit == 1   # every gradient element stored (no atomics): no zeroing needed after use
        use_parts = want_parts and nsplit == 1
        st = stats if stats is not None else self._dummy_stats
        items = self.wgrad_items(B, use_parts, clips)
        ls_part = self.parts[0][self.items[0]:self.items[0] + 1] if (use_parts and self.g_log_std is not None) else None
        ops.mlp_wgrad(items, nrt, nsplit, self.g_log_std, self.A, ls_part, float(clips[0] or -1.0), st, ent_coef,
                      kl_coef, self._mpart(B), nrt, bump)
        return use_parts

    def wgrad_items(self, B, parts=True, clips=(None, None)):
        """Item table of the weight-gradient launch (``mlp.hip`` mlp_wgrad_kernel, 8 int64 per 16 x 16 tile of every
        dW_l): operand block bases and strides, the gradient tile, its bias (first row of tiles), its sum-of-squares
        slot in :attr:`parts` and the clip applied before squaring; item 0 of a tower zeroes the tower's unused
        slots."""
        key = (B, bool(parts), clips)
        if key in self._witems:
            return self._witems[key]
        _, ws = self.desc(B)
        import struct
        recs = []
        wi = 0
        for t, tw in enumerate(self.towers):
            clip = float(clips[t] or -1.0)
            cbits = struct.unpack("<i", struct.pack("<f", clip))[0] & 0xFFFFFFFF
            local = 0
            first_unused = self.items[t] + (1 if t == 0 and self.g_log_std is not None else 0)
            for lay in tw:
                xs, dp = ws[wi], ws[wi + 1]
                wi += 2
                K, N = lay.in_features, lay.out_features
                gW = self._views(lay.kernel)[1]
                gb = self._views(lay.bias)[1]
                sx, sp = _nct(K) * 256, _nct(N) * 256
                for ti in range(_nct(K)):
                    for tj in range(_nct(N)):
                        ni, nj = min(16, K - 16 * ti), min(16, N - 16 * tj)
                        slot = self.parts[t].data_ptr() + 4 * local if parts else 0
                        zf = first_unused if (parts and local == 0) else 0
                        recs.append([xs.data_ptr() + 4 * 256 * ti, dp.data_ptr() + 4 * 256 * tj, sx | (sp << 32),
                                     ni | (nj << 8) | (N << 32), gW.data_ptr() + 4 * (16 * ti * N + 16 * tj),
                                     gb.data_ptr() + 4 * 16 * tj if ti == 0 else 0, slot, cbits | (zf << 32)])
                        local += 1
            assert local == self.items[t] and first_unused <= PARTS
        out = torch.tensor(recs, dtype=torch.int64).to(self.dev)
        self._witems[key] = out
        return out

    # ------------------------------------------------------------------------------------------- fused rollout
    def supports_fused_rollout(self, env):
        from ..envs.mujoco import MujocoShapeVecEnv
        return (isinstance(env, MujocoShapeVecEnv) and not self.discrete and self.A == LIN_ACT
                and self.D == LIN_OBS * env.frame_stack and env.frame_stack <= 3 and self.rollout_weights_in_lds()
                and [l.out_features for l in self.towers[0]] == [128, 128, 64, LIN_ACT])   # mlp_rollout_kernel shapes

    ROLLOUT_MAX_LDS = 150 * 1024
    ROLL_RB = 4   # envs per rollout workgroup (mlp.hip ROLL_RB: 4x4x1 MFMA tiles)

    def rollout_lds_bytes(self, wlds):
        """Dynamic LDS of mlp_rollout_kernel (layout in mlp.hip); ``wlds`` adds the staged actor weights + biases."""
        RB = self.ROLL_RB
        n = 2 * RB * _ld(self.D) + sum(RB * _ld(l.out_features) for l in self.towers[0])
        n += LIN_OBS * LIN_OBS + LIN_OBS * LIN_ACT + RB * LIN_OBS + RB * 16
        if wlds:
            n = (n + 3) // 4 * 4 + sum(l.out_features * _ld(l.in_features) + _ld(l.out_features) - 4
                                       for l in self.towers[0])
        return 4 * n

    def rollout_weights_in_lds(self):
        return self.rollout_lds_bytes(True) <= self.ROLLOUT_MAX_LDS

    def rollout_linear(self, env, st, key_shift, seed, stamps=None):
        """T steps of policy + env for the whole bank in one launch, then V(s) of all (T+1) N observations in one
        critic launch. Equal to T x (:meth:`policy_step` + ``env.step``) + :meth:`value` up to the actor's fp32
        summation order (4x4x1 tiles with the K range split over waves vs 16x16x4 tiles): same RNG keys and resets."""
        T, N = st.T, env.num_envs
        desc, _ = self.desc(None)
        wlds = self.rollout_weights_in_lds()
        _native.require().mlp_rollout(desc, self.rollout_lds_bytes(wlds), st.obs, st.actions, st.logp, st.entropy,
                                      st.rewards, st.dones, st.truncated, self.log_std, self.ac_scale, key_shift, seed,
                                      env.state, env.t, env.tg, env.ep_ret, env.ep_stats, env.env_ids, env.A, env.B,
                                      env.seed, env.max_episode_steps, env.frame_stack, wlds, stamps)
        self.value(st.obs.view((T + 1) * N, -1), st.values.view(-1))
