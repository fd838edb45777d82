#!/usr/bin/env python3
"""Regenerate scripts/exp/attn_exp.hip from csrc/mtq_attention.hip with s_memtime stamps per wave
(entry, prologue landed, loop done, epilogue done; per pass) for scripts/exp/bench_attn_exp.py."""
from pathlib import Path

R = Path(__file__).resolve().parents[2]
import subprocess, sys
src = "tensorrt-model-optimizer_amd/csrc/mtq_attention.hip"
# optional git revision: the copy built from that commit (A/B against the working tree product)
s = (subprocess.run(["git", "-C", str(R), "show", f"{sys.argv[1]}:{src}"], check=True, capture_output=True, text=True).stdout
     if len(sys.argv) > 1 else (R / src).read_text())


def sub(old, new):
    global s
    assert s.count(old) >= 1, old
    s = s.replace(old, new, 1)


sub('#include "mtq_device.hpp"\n', '#include "mtq_device.hpp"\n\n'
    '// measurement copy of csrc/mtq_attention.hip (scripts/exp/mk_attn_exp.py): s_memtime stamps per wave\n'
    '__device__ unsigned long long *g_st;\n'
    '__device__ __forceinline__ void stamp(int slot) {\n'
    '  unsigned long long *p = g_st;\n'
    '  if (p && (threadIdx.x & 63) == 0) p[((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + slot] = __builtin_amdgcn_s_memtime();\n'
    '}\n')
sub('unsigned char *__restrict__ Ks, unsigned char *__restrict__ Vs) {',
    'unsigned char *__restrict__ Ks, unsigned char *__restrict__ Vs, int sp) {\n  stamp(sp);')
sub('  __builtin_amdgcn_s_waitcnt(0x0F70);  // gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15\n  __syncthreads();\n',
    '  __builtin_amdgcn_s_waitcnt(0x0F70);  // gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15\n  __syncthreads();\n  stamp(sp + 1);\n')
sub('  // ---- o = acc / max(l, 1e-6); lane holds', '  stamp(sp + 2);\n  // ---- o = acc / max(l, 1e-6); lane holds')
sub('attn_tile<T, D, PQ, kStage>(a, b, h, kvh, t_long, Ks, Vs);', 'attn_tile<T, D, PQ, kStage>(a, b, h, kvh, t_long, Ks, Vs, 0);\n    stamp(3);')
sub('attn_tile<T, D, PQ, kStage>(a, b, h, kvh, pr, Ks, Vs);', 'attn_tile<T, D, PQ, kStage>(a, b, h, kvh, pr, Ks, Vs, 4);\n      stamp(7);')
sub('extern "C" int mtq_attention_fwd(',
    'namespace mtq {\nint host_check_launch() { return hipGetLastError() == hipSuccess ? 0 : -1; }\n}\n'
    'extern "C" int attn_exp_set_stamps(void *p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_st), &p, sizeof(p)) == hipSuccess ? 0 : -1; }\n'
    'extern "C" int attn_exp_fwd(')
(R / "scripts/exp/attn_exp.hip").write_text(s)
