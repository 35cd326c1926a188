"""Process-wide runtime settings of the HIP path: compute precision and the per-call
dropout seeds (counter-based masks need a distinct seed per op per step)."""
import itertools

import torch


class _Runtime:
    def __init__(self):
        self.compute_dtype = torch.bfloat16   # GEMM/attention operand dtype ("bf16" bench mode)
        self.flash_attention = True           # bf16 fused attention; False -> materialised GEMM+softmax
        # "fp8_attn" precision: attention forward on fp8 (e4m3) MFMA with per-tile power-of-two
        # scales, bf16 everywhere else (BASELINE config 5); backward = bf16 kernels on the fp8-rounded
        # q / k / v (straight-through)
        self.attn_fp8 = False
        # VAE ResnetBlock: GroupNorm+SiLU applied inside the halo conv's input staging (True) or as
        # a separate apply pass (False: tests compare the two)
        self.vae_gn_in_conv = True
        # dX of the LayerNorm-fed GEMMs in the compute dtype (autocast semantics) instead of fp32
        self.ln_dy_lowp = True
        # timm Mlp forward (bf16).  False: fc1 + GELU + dropout and fc2 + dropout + fp32 residual each in ONE
        # launch of the 8-wave GEMM (csrc/gemm8w.hip: two waves per SIMD, so one wave's epilogue runs beside
        # its partner's MFMAs).  True: bias-only GEMMs + one elementwise pass each (the route rounds 1-5
        # kept: at one wave per SIMD the fused epilogue was not hidden).  Same bits either way.
        self.mlp_split_epilogue = False
        # attention proj + proj_drop + residual (bf16) on the 8-wave GEMM's epilogue (the bf16 rounding of the
        # proj output before the dropout and the fp32 residual add, as autocast) instead of gemm_8ph's fused
        # epilogue (which kept the fp32 accumulator): 59-62 vs 72-75 us at B32 (profiles/r06/g8w_fused.txt)
        self.proj_8w = True
        # the remaining plain K-contiguous products (qkv forward, the Block's dX products, the DiffLoss MLP) on the
        # 8-wave GEMM instead of gemm_4w (uva_gemm8w_set; the same bits, tests/test_gemm8w_gpu.py): bench 263.9 /
        # 264.2 vs 262.3 / 263.7 samples/s, same box interleaved (profiles/r06/ab_gemm8w_plain.txt)
        self.gemm8w_plain = True
        self._gemm8w_plain_set = None
        # the proj / fc1 / fc2 dropout masks of a Block as keep-bit planes (one launch each per step) read by the
        # fused epilogues, instead of the counter hash per element inside them (the same bits).  Measured off:
        # the epilogue's plane-word loads expose their latency where the hash was issue-bound VALU (fc1 285-296
        # vs 253-271 us, bench 255.2 vs 257.7 samples/s same box, profiles/r06/g8w_planes.txt); kept tested
        self.drop_planes = False
        # the qkv bias gradient from the attention backward kernels' epilogues (no column-sum pass over dqkv)
        self.attn_bias_grad = True
        # norm2's LayerNorm backward also emits the proj_drop backward + proj bias gradient (one pass over dx)
        self.ln_bwd_drop = True
        # Mlp backward: dropout + GELU' (+ the fc1 bias gradient) in the epilogue of fc2's dX product (8-wave
        # GEMM, EPI 3) instead of dX GEMM -> act_bwd_bias (one [M, 3072] bf16 round trip less per Block)
        self.act_bwd_in_gemm = True
        # the same for the DiffLoss SimpleMLPAdaLN trunk (SiLU, W = 1024) on gemm_8ph's dX epilogue: measured
        # slower there (128.4 vs 125.8 ms/step, one wave per SIMD); kept off, the mode tested
        self.trunk_act_bwd_in_gemm = False
        self._seed_base = 0x5EED
        self._ctr = itertools.count()
        # attention dropout masks: per Block the (B, N, H, p) of its last training forward, and the
        # masks generated ahead of time on a side stream (overlapping the VAE encode)
        self.attn_prefetch = True
        # VAE encoder level at whose start the keep-mask planes are launched on the side stream (0: before
        # the encode).  The planes' VALU-bound kernels took CU time from the level-0 GN convs (237 us per
        # launch under them vs 78 us alone); from level 2 on the convs are smaller
        self.attn_prefetch_level = 2
        self._prefetch_pending = None
        # transposed bf16 weights of the Blocks' dX products, built on the side stream with the masks
        self.weight_t_prefetch = True
        self._weight_t_params = []
        self._attn_shapes = {}
        self._attn_ready = {}
        self._side = None
        # cross-Block fusion of the fc2 dropout backward into the NEXT Block's norm1 backward: a Block's output
        # (data_ptr) -> (the output itself, p, seed, fc2.bias) while a training forward is in flight; the
        # consumer Block's backward leaves (dX tensor it produced, bf16(drop(dX))) under the seed
        self._drop_pending = {}
        self._drop_ready = {}
        # bumped whenever HIP kernels rewrite parameters in place (optimizer / EMA steps): caches
        # keyed on parameters (non-static compute shadows, the sampler's captured graphs) compare it
        self.param_gen = 0

    def set_precision(self, name):
        name = str(name).lower()
        self.attn_fp8 = False
        if name in ("fp32", "float32", "no"):
            self.compute_dtype = torch.float32
        elif name in ("bf16", "bfloat16", "fp16"):
            # fp16 autocast of the reference maps to bf16 MFMA here (same 16-bit storage,
            # wider exponent; no GradScaler needed)
            self.compute_dtype = torch.bfloat16
        elif name in ("fp8_attn", "fp8"):
            self.compute_dtype = torch.bfloat16
            self.attn_fp8 = True
        else:
            raise ValueError(f"unknown precision {name}")

    def begin_forward(self):
        """a new MAR forward: hand-offs of the previous step that found no consumer are dropped"""
        self._drop_pending.clear()
        self._drop_ready.clear()
        if self._gemm8w_plain_set is not self.gemm8w_plain:
            from .native import ops
            ops.gemm8w_set(int(self.gemm8w_plain), -2)
            self._gemm8w_plain_set = self.gemm8w_plain

    def bump_params(self):
        self.param_gen += 1

    def seed(self, base):
        self._seed_base = int(base)
        self._ctr = itertools.count()

    def next_seed(self):
        return (self._seed_base * 0x9E3779B97F4A7C15 + next(self._ctr) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF


    # ---- attention dropout-mask prefetch ------------------------------------------------
    def note_attn_shape(self, key, shape):
        self._attn_shapes[key] = shape

    def arm_attn_prefetch(self, device):
        """schedule prefetch_attn_masks for the VAE encode that follows: fired by the encoder at the start
        of level attn_prefetch_level (vae/vaekl.py moments_nhwc), or right away for level 0"""
        if self.attn_prefetch_level <= 0:
            self.prefetch_attn_masks(device)
        else:
            self._prefetch_pending = device

    def fire_attn_prefetch(self, level=None):
        """launch an armed prefetch (level None: unconditionally, e.g. after an encode that had fewer levels)"""
        dev = self._prefetch_pending
        if dev is not None and (level is None or level >= self.attn_prefetch_level):
            self._prefetch_pending = None
            self.prefetch_attn_masks(dev)

    def prefetch_attn_masks(self, device):
        """side-stream work launched under the VAE encode: the attention keep-mask planes of every known Block,
        then the transposed bf16 weight copies the Blocks' dX products use (registered by the policy)"""
        self._prefetch_masks(device)
        if self.weight_t_prefetch and self._weight_t_params and self._side is not None:
            from .model.autoregressive.functional import prefetch_weight_t
            self._side.wait_stream(torch.cuda.current_stream(device))
            prefetch_weight_t(self._weight_t_params, self._side)

    def _prefetch_masks(self, device):
        """Generate every known Block's attention keep-mask planes for this step on a side stream,
        so the VALU-bound mask kernels run under the (MFMA-bound) VAE encode that precedes the MAR.
        Each Block waits on its own event before its attention forward reads the planes."""
        if not (self.attn_prefetch and self._attn_shapes and torch.cuda.is_available()):
            return
        from .native import ops
        if self._side is None:
            self._side = torch.cuda.Stream(device=device)
        main = torch.cuda.current_stream(device)
        self._side.wait_stream(main)
        ready = {}
        for key, (B, N, H, p) in self._attn_shapes.items():
            seed = self.next_seed()
            mask = ops.attn_mask_alloc(B, N, H, device)  # allocated in main-stream order
            with torch.cuda.stream(self._side):
                ops.attn_dropmask(B, N, H, p, seed, device, out=mask)
            ev = torch.cuda.Event()
            ev.record(self._side)
            mask.record_stream(self._side)
            ready[key] = ((B, N, H, p), seed, mask, ev)
        self._attn_ready = ready

    def take_attn_mask(self, key, shape):
        """-> (seed, mask) prefetched for this Block and shape (the current stream now waits for
        it), or None."""
        hit = self._attn_ready.pop(key, None)
        if hit is None or hit[0] != shape:
            return None
        torch.cuda.current_stream().wait_event(hit[3])
        return hit[1], hit[2]


RT = _Runtime()


def cdt():
    return RT.compute_dtype
