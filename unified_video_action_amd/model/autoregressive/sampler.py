"""Reverse-diffusion sampler of the action head (inference path).

Reference: DiffActLoss.sample (diffusion_action_loss.py:168-232) ->
gen_diffusion.p_sample_loop (gaussian_diffusion.py:395-492) over the spaced cosine
schedule (create_diffusion(timestep_respacing=act_diff_testing_steps), respace.py:65-130),
with the SimpleMLPAdaLN net (diffusion_loss.py:192-283) as the eps / variance model.

MI355X layout of one sampling call over R = B*16 action rows and S spaced steps:
  * everything that depends only on (cond, t) is hoisted out of the step loop: the
    cond embedding once, the S timestep embeddings once, and the adaLN modulation of
    every res block and the final layer for ALL steps as ONE [S*R, W] x [W, (3d+2)W]
    GEMM (the sampler's dominant FLOPs; per step it would be S launches at M=R);
  * the step loop is what is left: input_proj, d x (adaLN-LN, fc1 + SiLU, fc2 + gate +
    residual) and LN-modulate + final linear, the linears as few-row fused kernels
    (uva_sampler_linear: 32x64 tiles over the full K, weights preloaded into registers, or for
    few rows 32x16 tiles with K split over 8 waves; optional LayerNorm in the A staging -- used
    for the final layer, and for fc1 at few rows),
    and the fused p_sample update kernel (uva_p_sample_step) -- replayed from a captured HIP graph after one eager step
    (which also settles the per-shape GEMM route choices before capture).
No autograd and no backward residues (the training trunk's aux tensors) are produced.
"""

import warnings

import torch

from ...native import ops
from ...runtime import RT, cdt
from .diffusion import SamplingSchedule, timestep_freqs
from .functional import F32, compute_weight

_SCHED = {}


def sampling_schedule(respacing, T=1000):
    key = (T, str(respacing))
    if key not in _SCHED:
        _SCHED[key] = SamplingSchedule(T, str(respacing))
    return _SCHED[key]


class ActionSampler:
    """One p_sample_loop over the SimpleMLPAdaLN `net` conditioned on c [R, z] (fp32)."""

    MOD_BYTES_CAP = 16 << 30  # all-step modulation table above this is computed per step
    # few-row kernels re-read the weights once per 32-row block: beyond ~1k rows (video sampling,
    # B*1024 tokens) the general 256x256-tile GEMMs are the right tool
    FUSED_MAX_ROWS = 1024

    def __init__(self, net, respacing="100", use_graph=True, use_fused=True, clip_denoised=True,
                 use_persistent=True):
        self.net = net
        # few rows (R <= 16: action sampling at B = 1): the whole loop as ONE persistent launch
        # (uva_sampler_persistent) instead of the captured ~15 launches per step
        self.use_persistent = use_persistent
        self.clip = clip_denoised  # action head: True (diffusion_action_loss.py:218); video head: False
        self.sched = sampling_schedule(respacing)
        self.use_graph = use_graph
        self.use_fused = use_fused  # few-row fused LN+linear kernels (bf16 compute, width <= 1024)
        # LN inside fc1's A staging re-normalises the rows once per column block: at B=32 (512 rows)
        # measured slower than the separate LN kernel (27.8 vs 26.0 ms / loop); at few rows (B=1:
        # 16 rows) the separate LN launch costs more than the redundant re-normalisation
        self.fuse_ln_rows = 64

    def __deepcopy__(self, memo):
        """copies (the reference's deepcopy'd EMA policy) start without the cached buffers / graph."""
        import copy
        new = ActionSampler.__new__(ActionSampler)
        memo[id(self)] = new
        for k, v in self.__dict__.items():
            if k != "_cache":
                new.__dict__[k] = copy.deepcopy(v, memo)
        return new

    # ---- hoisted conditioning -------------------------------------------------------------
    def _weights(self):
        net = self.net
        blocks = [b.trunk_params() for b in net.res_blocks]
        fl = net.final_layer.trunk_params()
        wcat = torch.cat([compute_weight(b[0]) for b in blocks] + [compute_weight(fl[0])], 0).contiguous()
        bcat = torch.cat([b[1].detach() for b in blocks] + [fl[1].detach()], 0).float().contiguous()
        return blocks, fl, wcat, bcat

    def _time_embed(self, dev):
        te = self.net.time_embed
        tmap = torch.tensor([s[1] for s in self.sched.steps], dtype=torch.int64, device=dev)
        f = torch.empty(tmap.numel(), te.frequency_embedding_size, dtype=cdt(), device=dev)
        ops.timestep_features(tmap, timestep_freqs(dev), f)
        h = torch.empty(tmap.numel(), te.mlp[0].weight.shape[0], dtype=cdt(), device=dev)
        ops.linear(f, compute_weight(te.mlp[0].weight), h, bias=te.mlp[0].bias.detach(), act="silu")
        out = torch.empty(tmap.numel(), te.mlp[2].weight.shape[0], dtype=F32, device=dev)
        ops.linear(h, compute_weight(te.mlp[2].weight), out, bias=te.mlp[2].bias.detach())
        return out  # [S, W], row k = step k of the loop

    def _modulation(self, c, st):
        """sy_k = SiLU(cond_embed(c) + t_emb_k);  mod[k] = sy_k @ wcat^T + bcat -> st["mod"] [S, R, (3d+2)W]
        (or st["sy"] only, when the all-step table is over MOD_BYTES_CAP)."""
        net = self.net
        R = c.shape[0]
        W = net.model_channels
        dev = c.device
        yc = torch.empty(R, W, dtype=F32, device=dev)
        ops.linear(c.to(cdt()).contiguous(), compute_weight(net.cond_embed.weight), yc,
                   bias=net.cond_embed.bias.detach())
        te = self._time_embed(dev)
        S = te.shape[0]
        y = yc[None] + te[:, None]  # [S, R, W] fp32 (t + c, diffusion_loss.py:276-278)
        ops.act_fwd(y, st["sy"], "silu")
        del y
        if st["mod"] is not None:
            ncol = st["wcat"].shape[0]
            ops.linear(st["sy"].reshape(S * R, W), st["wcat"], st["mod"].reshape(S * R, ncol), bias=st["bcat"])

    # ---- one reverse step (captured) --------------------------------------------------------
    def _step(self, k, st):
        net = self.net
        R, C, W = st["R"], st["C"], net.model_channels
        blocks, fl, mod_all = st["blocks"], st["fl"], st["mod"]
        if mod_all is None:
            mod = st["mod_buf"]
            ops.linear(st["sy"][k], st["wcat"], mod, bias=st["bcat"])
        else:
            mod = mod_all[k]
        x = st["h0"]
        ops.linear(st["x_net"], compute_weight(net.input_proj.weight), x, bias=net.input_proj.bias.detach())
        if st["fused"]:
            for i, (modw, modb, w1, b1, w2, b2, lnw, lnb) in enumerate(blocks):
                m = mod[:, 3 * W * i:3 * W * (i + 1)]
                if R <= self.fuse_ln_rows:
                    ops.sampler_linear(x, compute_weight(w1), st["a"], bias=b1.detach(), act="silu", ln=True,
                                       lnw=lnw.detach(), lnb=lnb.detach(), shift=m[:, :W], scale=m[:, W:2 * W])
                else:
                    ops.layernorm_fwd(x, lnw.detach(), lnb.detach(), st["h"], st["mean"], st["rstd"],
                                      scale=m[:, W:2 * W], shift=m[:, :W], ldm=mod.shape[1])
                    ops.sampler_linear(st["h"], compute_weight(w1), st["a"], bias=b1.detach(), act="silu")
                xn = st["h1"] if x is st["h0"] else st["h0"]
                ops.sampler_linear(st["a"], compute_weight(w2), xn, bias=b2.detach(), gate=m[:, 2 * W:3 * W],
                                   residual=x)
                x = xn
            fm = mod[:, 3 * W * len(blocks):]
            ops.sampler_linear(x, compute_weight(fl[2]), st["out"], bias=fl[3].detach(), ln=True,
                               shift=fm[:, :W], scale=fm[:, W:2 * W])
        else:
            self._step_unfused(x, mod, st)
        coef = list(self.sched.steps[k][2]) + [st["temperature"]]
        ops.p_sample_step(st["out"], st["x"], st["noise"][k], coef, st["x"], st["x_net"], clip=self.clip)

    def _step_unfused(self, x, mod, st):
        """general-route step body (fp32 parity mode, or widths over the fused kernel's K limit)."""
        W = self.net.model_channels
        blocks, fl, ncol = st["blocks"], st["fl"], mod.shape[1]
        for i, (modw, modb, w1, b1, w2, b2, lnw, lnb) in enumerate(blocks):
            m = mod[:, 3 * W * i:3 * W * (i + 1)]
            ops.layernorm_fwd(x, lnw.detach(), lnb.detach(), st["h"], st["mean"], st["rstd"],
                              scale=m[:, W:2 * W], shift=m[:, :W], ldm=ncol)
            ops.linear(st["h"], compute_weight(w1), st["a"], bias=b1.detach(), act="silu")
            xn = st["h1"] if x is st["h0"] else st["h0"]
            ops.linear(st["a"], compute_weight(w2), xn, bias=b2.detach(), gate=m[:, 2 * W:3 * W], residual=x)
            x = xn
        fm = mod[:, 3 * W * len(blocks):]
        ops.layernorm_fwd(x, None, None, st["h"], st["mean"], st["rstd"], scale=fm[:, W:2 * W], shift=fm[:, :W],
                          ldm=ncol)
        ops.linear(st["h"], compute_weight(fl[2]), st["out"], bias=fl[3].detach())

    def _state(self, R, C, dev, temperature):
        """Persistent step buffers (+ captured graph) per (rows, channels, dtype, weights)."""
        net = self.net
        cd = cdt()
        # RT.param_gen: the optimizer / EMA kernels rewrite weights without bumping _version, and the
        # captured graph and the concatenated modulation weights (wcat / bcat) must follow them
        sig = (R, C, str(cd), float(temperature), str(dev), self.use_fused, self.use_persistent, RT.param_gen,
               tuple((p.data_ptr(), p._version) for p in net.parameters()))
        cache = getattr(self, "_cache", None)
        if cache is not None and cache["sig"] == sig:
            return cache
        W = net.model_channels
        S = self.sched.S
        blocks, fl, wcat, bcat = self._weights()
        ncol = wcat.shape[0]
        per_step = S * R * ncol * (torch.finfo(cd).bits // 8) > self.MOD_BYTES_CAP
        st = dict(sig=sig, R=R, C=C, blocks=blocks, fl=fl, wcat=wcat, bcat=bcat, temperature=float(temperature),
                  sy=torch.empty(S, R, W, dtype=cd, device=dev),
                  mod=None if per_step else torch.empty(S, R, ncol, dtype=cd, device=dev),
                  mod_buf=torch.empty(R, ncol, dtype=cd, device=dev) if per_step else None,
                  x=torch.empty(R, C, dtype=F32, device=dev), noise=torch.empty(S, R, C, dtype=F32, device=dev),
                  x_net=torch.empty(R, C, dtype=cd, device=dev),
                  h0=torch.empty(R, W, dtype=F32, device=dev), h1=torch.empty(R, W, dtype=F32, device=dev),
                  h=torch.empty(R, W, dtype=cd, device=dev), a=torch.empty(R, W, dtype=cd, device=dev),
                  mean=torch.empty(R, dtype=F32, device=dev), rstd=torch.empty(R, dtype=F32, device=dev),
                  out=torch.empty(R, 2 * C, dtype=F32, device=dev), graph=None,
                  fused=self.use_fused and cd == torch.bfloat16 and W in (256, 512, 1024) and R <= self.FUSED_MAX_ROWS)
        st["persist"] = (self.use_persistent and st["fused"] and st["mod"] is not None and R <= 16 and W == 1024
                         and len(blocks) == 6 and C <= 16 and dev.type == "cuda"
                         and ops.sampler_persistent_fits(dev))
        if st["persist"]:
            # weights stacked per kind (one base pointer each), coefficient table [S, 8] on the device
            st["pack"] = dict(
                w1=torch.stack([compute_weight(b[2]) for b in blocks]).contiguous(),
                b1=torch.stack([b[3].detach().float() for b in blocks]).contiguous(),
                w2=torch.stack([compute_weight(b[4]) for b in blocks]).contiguous(),
                b2=torch.stack([b[5].detach().float() for b in blocks]).contiguous(),
                lnw=torch.stack([b[6].detach().float() for b in blocks]).contiguous(),
                lnb=torch.stack([b[7].detach().float() for b in blocks]).contiguous(),
                win=compute_weight(net.input_proj.weight).contiguous(),
                bin=net.input_proj.bias.detach().float().contiguous(),
                wf=compute_weight(fl[2]).contiguous(), bfin=fl[3].detach().float().contiguous())
            st["coef"] = torch.tensor([list(self.sched.steps[k][2]) + [float(temperature)] for k in range(S)],
                                      dtype=F32, device=dev)
            st["work"] = ops.sampler_persistent_workspace(W, dev)
            st["xo"] = torch.empty(R, C, dtype=F32, device=dev)
        self._cache = st
        return st

    @torch.no_grad()
    def __call__(self, c, noise, step_noise, temperature=1.0):
        """c [R, z] fp32 cond, noise [R, C] x_T, step_noise [S, R, C] -> x_0 [R, C] fp32."""
        dev = c.device
        R, C = noise.shape
        S = self.sched.S
        if step_noise.shape != (S, R, C):
            raise ValueError(f"step_noise {tuple(step_noise.shape)} != {(S, R, C)}")
        if c.shape[0] != R:
            raise ValueError(f"cond rows {c.shape[0]} != noise rows {R}")
        st = self._state(R, C, dev, temperature)
        self._modulation(c, st)
        if st["persist"]:
            ops.sampler_persistent(st["pack"], st["mod"], st["coef"], step_noise.contiguous(), noise.contiguous(),
                                   st["xo"], st["work"], clip=self.clip)
            # the launch relies on its 64 workgroups being co-resident; if any hand-off wait ran into
            # its spin bound (CUs held by other streams, a partitioned device) the kernel wrote NaN and
            # set the flag: recompute this call on the captured-graph route and stop using the
            # persistent kernel for this state (one 4-byte read, ~tens of us at B = 1)
            if ops.sampler_persistent_status(st["work"]) == 0:
                return st["xo"].clone()
            warnings.warn("persistent action sampler gave up on a hand-off (workgroups not co-resident); "
                          "recomputing on the captured-graph route", RuntimeWarning)
            st["persist"] = False
            self.persistent_giveups = getattr(self, "persistent_giveups", 0) + 1
        st["x"].copy_(noise)
        st["x_net"].copy_(noise)
        st["noise"].copy_(step_noise)
        self._step(0, st)  # eager: settles GEMM routes and workspaces before capture
        if S > 1 and self.use_graph and dev.type == "cuda":
            if st["graph"] is None:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for k in range(1, S):
                        self._step(k, st)
                st["graph"] = g
                # capture records without executing: run the captured steps once now
            st["graph"].replay()
        else:
            for k in range(1, S):
                self._step(k, st)
        return st["x"].clone()
