"""Diagnostic builds of the GN halo conv (timing only; results are WRONG by construction): each
variant patches a copy of csrc/conv.hip, compiles it, and links abx/diag_<name>.so from the in-tree
objects with conv.o replaced.  Run the timings with tools/conv_diag.sh on the GPU box."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "unified_video_action_amd", "csrc")
OBJ = os.path.join(ROOT, "unified_video_action_amd", "build_obj")
AB = os.path.join(ROOT, "abx")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics", "-Wno-unused-result",
         "-I" + CSRC] + os.environ.get("DIAG_FLAGS", "").split()

ANCHOR = "  const int pid = ch_xcd_remap(blockIdx.x, nblk);"
VARIANTS = {
    "base": [],
    # GN apply without SiLU (no exp / rcp)
    "nosilu": [("if (gn_silu) {", "if (false) {")],
    # register-B weight loads always from step 0's offset (L1/L2-hot lines: the weight stream's latency)
    "bhot": [("const int soff = __builtin_amdgcn_readfirstlane((tap * Ci + cc * 64) * 2);",
              "const int soff = 0;")],
    # no halo restaging at the chunk boundary (the chunk-1 MFMAs read stale LDS)
    # no epilogue (MFMA results folded into one improbable-condition store)
    "noepi": [("    ch_lds_barrier();  // the epilogue's LDS image overlays the halo buffers",
               "    ch_lds_barrier();\n    { float sm = 0.f;\n      for (int f = 0; f < G::FM; ++f) for (int g = 0; g < G::FN; ++g) sm += acc[f][g][0] + acc[f][g][3];\n"
               "      if (sm == 1.2345e-30f) out[tid] = (bf16)sm;\n      return; }")],
    # register-epilogue form without its epilogue
    "rnoepi": [("    // ---- register epilogue: + residual",
                "    { float sm = 0.f;\n      for (int f = 0; f < G::FM; ++f) for (int g = 0; g < G::FN; ++g) sm += acc[f][g][0] + acc[f][g][3];\n"
                "      if (sm == 1.2345e-30f) out[tid] = (bf16)sm;\n      return; }\n    // ---- register epilogue: + residual")],
    # register epilogue without the GroupNorm partial sums
    "rnogn": [("    if (gn_part) {\n      const int gsz = Co / 32;", "    if (false) {\n      const int gsz = Co / 32;"),
              ("        if (gn_part) {\n          const uint2 u", "        if (false) {\n          const uint2 u")],
    # register epilogue without the output stores (GN sums kept)
    "rnost": [("        *(bf16x4*)(out + (pix0 + (long long)f * W) * Co + c0 + g * 16) = o;", "")],
    # MFMA loop with the weight fragment outer
    "gouter": [("""          for (int f = 0; f < G::FM; ++f)
#pragma unroll
            for (int g = 0; g < G::FN; ++g)
              acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[cur][ks][g], fa[ks][f], acc[f][g], 0, 0, 0);""",
                """          for (int g = 0; g < G::FN; ++g)
#pragma unroll
            for (int f = 0; f < G::FM; ++f)
              acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[cur][ks][g], fa[ks][f], acc[f][g], 0, 0, 0);""")],
    # accumulators not seeded with the bias
    "zinit": [("    if (RB && bias) {", "    if (false) {")],
    # operands in the pixel-major order (wrong layout for the epilogue; timing only)
    "aorder": [("mfma_f32_16x16x32_bf16(bq[cur][ks][g], fa[ks][f], acc[f][g], 0, 0, 0)",
                "mfma_f32_16x16x32_bf16(fa[ks][f], bq[cur][ks][g], acc[f][g], 0, 0, 0)")],
    # attention dropout planes without the hash (timing of the step without the mask cost)
    "maskfree": [("    const uint32_t hv = drop_hash(key, pair0 + j);", "    const uint32_t hv = (uint32_t)(pair0 + j) * 0x9E3779B1u;")],
    # the second co-resident workgroup of each CU (dispatch slots 256..511) starts ~half a tile late
    "stag2": [(ANCHOR, "  if (blockIdx.x >= 256 && blockIdx.x < 512) for (int i = 0; i < 2; ++i) __builtin_amdgcn_s_sleep(127);\n" + ANCHOR)],
    "stag4": [(ANCHOR, "  if (blockIdx.x >= 256 && blockIdx.x < 512) for (int i = 0; i < 4; ++i) __builtin_amdgcn_s_sleep(127);\n" + ANCHOR)],
    "stag8": [(ANCHOR, "  if (blockIdx.x >= 256 && blockIdx.x < 512) for (int i = 0; i < 8; ++i) __builtin_amdgcn_s_sleep(127);\n" + ANCHOR)],
    # A fragments read from LDS at tap 0 of each chunk only (later taps reuse them): the A-read cost
    "noA": [("""        bf16x8 fa[2][G::FM];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int f = 0; f < G::FM; ++f)
            fa[ks][f] =""", """        if (tap == 0)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int f = 0; f < G::FM; ++f)
            fa[ks][f] ="""),
            ("""    for (int cc = 0; cc < nch; ++cc) {
      const bf16* hcur = halo + (cc & 1) * G::HALO_ELEMS + abase;""", """    bf16x8 fa[2][G::FM];
    for (int cc = 0; cc < nch; ++cc) {
      const bf16* hcur = halo + (cc & 1) * G::HALO_ELEMS + abase;""")],
    # the same, A fragments re-read at taps 0 and 4 (half the LDS A traffic)
    "halfA": [("""        bf16x8 fa[2][G::FM];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int f = 0; f < G::FM; ++f)
            fa[ks][f] =""", """        if ((tap & 1) == 0)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int f = 0; f < G::FM; ++f)
            fa[ks][f] ="""),
            ("""    for (int cc = 0; cc < nch; ++cc) {
      const bf16* hcur = halo + (cc & 1) * G::HALO_ELEMS + abase;""", """    bf16x8 fa[2][G::FM];
    for (int cc = 0; cc < nch; ++cc) {
      const bf16* hcur = halo + (cc & 1) * G::HALO_ELEMS + abase;""")],
    # persistent sampler: hand-off waits skipped (results wrong; the latency of the waits)
    "ps_nowait": [("      if (__hip_atomic_load((gu32*)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;",
                   "      break;")],
    # persistent sampler: exchanged rows not re-loaded (stale registers / LDS; latency of the sc1 loads)
    "ps_noload": [("        if (r < R)\n          v = __builtin_bit_cast", "        if (r < 0)\n          v = __builtin_bit_cast"),
                  ("        const u32x4v v = __builtin_amdgcn_raw_buffer_load_b128(rs_ha, (row * W + c8) * 2, 0, PS_SC1);\n        *(u32x4v*)(sA + row * PS_LDA + c8) = v;",
                   "        (void)row; (void)c8;")],
    # persistent sampler: no publish (counter adds skipped) AND no waits
    "ps_nosync": [("      if (__hip_atomic_load((gu32*)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;",
                   "      break;"),
                  ("  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");  // the storing wave's sc1 stores have left\n  if ((threadIdx.x & 63) == 0)",
                   "  if (false)")],
    # persistent sampler: s_memtime stamps of workgroup 0 / thread 0 at every phase point of step 50,
    # written at work + 1024 (tools/ps_stamps.py reads them); the workspace header grows to 8 KB
    "ps_stamps": [("  return 256 + 2LL * PS_R * W * 4 + (long long)PS_R * W * 2;", "  return 8192 + 2LL * PS_R * W * 4 + (long long)PS_R * W * 2;"),
                  ("  p.hx = (float*)((char*)work + 256);", "  p.hx = (float*)((char*)work + 8192);"),
                  ("  p.ha = (bf16*)((char*)work + 256 + 2LL * PS_R * W * 4);", "  p.ha = (bf16*)((char*)work + 8192 + 2LL * PS_R * W * 4);"),
                  ("  for (int k = 0; k < p.S; ++k) {\n    const unsigned target", "  unsigned long long* stp = (unsigned long long*)((char*)p.cnt + 1024);\n  int sti = 0;\n#define STAMP() do { if (blockIdx.x == 0 && tid == 0 && k == 50) stp[sti++] = __builtin_amdgcn_s_memtime(); } while (0)\n  for (int k = 0; k < p.S; ++k) {\n    STAMP();\n    const unsigned target"),
                  ("#pragma unroll 1\n    for (int blk = 0; blk < D; ++blk) {", "    STAMP();\n#pragma unroll 1\n    for (int blk = 0; blk < D; ++blk) {"),
                  ("        ps_wait(p.cnt + 2 * blk - 1, target, p.err);\n        load_h((blk - 1) & 1);\n        res_from_hx((blk - 1) & 1);",
                   "        ps_wait(p.cnt + 2 * blk - 1, target, p.err);\n        STAMP();\n        load_h((blk - 1) & 1);\n        res_from_hx((blk - 1) & 1);"),
                  ("      ln_mod(true);\n      __syncthreads();\n      mma(bw, 0);", "      ln_mod(true);\n      __syncthreads();\n      STAMP();\n      mma(bw, 0);"),
                  ("        ps_publish(p.cnt + 2 * blk);\n      }", "        ps_publish(p.cnt + 2 * blk);\n      }\n      STAMP();"),
                  ("      ps_wait(p.cnt + 2 * blk, target, p.err);\n", "      ps_wait(p.cnt + 2 * blk, target, p.err);\n      STAMP();\n"),
                  ("        ps_publish(p.cnt + 2 * blk + 1);\n      }", "        ps_publish(p.cnt + 2 * blk + 1);\n      }\n      STAMP();"),
                  ("      ps_wait(p.cnt + 2 * D - 1, target, p.err);\n      load_h((D - 1) & 1);", "      ps_wait(p.cnt + 2 * D - 1, target, p.err);\n      STAMP();\n      load_h((D - 1) & 1);")],
    # GN + SiLU with scalar f32 VALU (the packed v_pk_* forms cost extra issue beside MFMAs)
    "gnscalar": [("""#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            const f32x2 x = {(float)v[j], (float)v[j + 1]};
            f32x2 u = x * (f32x2){gsc[j], gsc[j + 1]} + (f32x2){gsh[j], gsh[j + 1]};
            if (gn_silu) {
              const f32x2 t = u * (f32x2){-1.4426950408889634f, -1.4426950408889634f};
              const f32x2 d = (f32x2){__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + (f32x2){1.f, 1.f};
              u = u * (f32x2){__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
            }
            v[j] = (bf16)u.x;
            v[j + 1] = (bf16)u.y;
          }""", """#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float u = __builtin_fmaf((float)v[j], gsc[j], gsh[j]);
            if (gn_silu) {
              const float d = __builtin_amdgcn_exp2f(u * -1.4426950408889634f) + 1.f;
              u = u * __builtin_amdgcn_rcpf(d);
            }
            v[j] = (bf16)u;
          }""")],
    "nostage": [("        halo_store((cc + 1) & 1);\n        ch_lds_barrier();", "        ch_lds_barrier();")],
}


FILES = {"maskfree": "attention.hip", "ps_nowait": "sampler.hip", "ps_noload": "sampler.hip",
         "ps_nosync": "sampler.hip", "ps_stamps": "sampler.hip"}


def build(name, subs, whole=None):
    """whole: path of a complete replacement for the source file (an A/B of a rewritten kernel)."""
    fn = FILES.get(name, "conv.hip")
    src = open(whole or os.path.join(CSRC, fn)).read()
    for a, b in subs:
        assert a in src, (name, a)
        src = src.replace(a, b)
    tmp = os.path.join(CSRC, f"_diag_{name}.hip")
    open(tmp, "w").write(src)
    try:
        obj = os.path.join(AB, f"{fn[:-4]}_{name}.o")
        subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + ["-c", tmp, "-o", obj], check=True)
    finally:
        os.remove(tmp)
    objs = [os.path.join(OBJ, f) for f in sorted(os.listdir(OBJ)) if f.endswith(".o") and f != fn[:-4] + ".o"] + [obj]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    os.path.join(AB, f"diag_{name}.so")] + objs, check=True)
    os.remove(obj)


if __name__ == "__main__":
    os.makedirs(AB, exist_ok=True)
    if len(sys.argv) == 4 and sys.argv[1] == "--file":  # --file NAME PATH: conv.hip replaced by PATH
        build(sys.argv[2], [], whole=sys.argv[3])
        print("built", sys.argv[2])
        sys.exit(0)
    for n in (sys.argv[1:] or VARIANTS):
        build(n, VARIANTS[n])
        print("built", n)
