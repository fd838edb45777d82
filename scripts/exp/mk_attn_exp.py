#!/usr/bin/env python3
"""Regenerate scripts/exp/attn_exp.hip from csrc/mtq_attention.hip with s_memtime stamps per wave
(entry, prologue landed, loop done, epilogue done; per pass) for scripts/exp/bench_attn_exp.py."""
import re
from pathlib import Path

R = Path(__file__).resolve().parents[2]
import subprocess, sys
src = "tensorrt-model-optimizer_amd/csrc/mtq_attention.hip"
# optional git revision: the copy built from that commit (A/B against the working tree product)
s = (subprocess.run(["git", "-C", str(R), "show", f"{sys.argv[1]}:{src}"], check=True, capture_output=True, text=True).stdout
     if len(sys.argv) > 1 and sys.argv[1] != "-" else (R / src).read_text())


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
s = re.sub(r"(unsigned char \*__restrict__ Ks, unsigned char \*__restrict__ Vs)([^)]*)\) \{",
           r"\1\2, int sp) {\n  stamp(sp);", s, count=1)
sub('  __builtin_amdgcn_s_waitcnt(0x0F70);  // gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15\n  __syncthreads();\n',
    '  __builtin_amdgcn_s_waitcnt(0x0F70);  // gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15\n  __syncthreads();\n  stamp(sp + 1);\n')
sub('  // ---- o = acc / max(l, 1e-6); lane holds', '  stamp(sp + 2);\n  // ---- o = acc / max(l, 1e-6); lane holds')
s = re.sub(r"(attn_tile<T, D, PQ, kStage>\(a, b, h, kvh, t_long, Ks, Vs)([^;]*)\);", r"\1\2, 0);\n    stamp(3);", s, count=1)
s = re.sub(r"(attn_tile<T, D, PQ, kStage>\(a, b, h, kvh, pr, Ks, Vs)([^;]*)\);", r"\1\2, 4);\n      stamp(7);", s, count=1)
sub('extern "C" int mtq_attention_fwd(',
    'namespace mtq {\nint host_check_launch() { return hipGetLastError() == hipSuccess ? 0 : -1; }\n}\n'
    'extern "C" int attn_exp_set_stamps(void *p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_st), &p, sizeof(p)) == hipSuccess ? 0 : -1; }\n'
    'extern "C" int attn_exp_fwd(')
out = sys.argv[2] if len(sys.argv) > 2 else "attn_exp"  # the library's entry points get this prefix
s = s.replace("attn_exp_set_stamps", f"{out}_set_stamps").replace("attn_exp_fwd", f"{out}_fwd")
(R / "scripts/exp" / f"{out}.hip").write_text(s)
