#!/usr/bin/env python3
"""Generate the K loop of the AWQ search kernel `awq_search_w4_kernel` (csrc/mtq_awq_gemm.hip) as one
inline-asm statement per input type: tensorrt-model-optimizer_amd/csrc/mtq_awq_w4.inc (committed;
tests/test_awq_w4_generated.py checks it is this script's output).

Schedule (one wave per SIMD, the shape hipBLASLt runs, written at the instruction level because
hipcc's waits collapse its prefetch; DESIGN.md §4e, measured in scripts/exp/awq_w4asm.hip):
* 4 waves per 256 x 256 output tile, a 128 x 128 block per wave (2 x 2), 64 16x16 fp32
  accumulators in a[0:255] (v_mfma_f32_16x16x32_{bf16,f16}, the W fragment as the A operand, so a
  lane holds out[m][n .. n+3] as the r03 kernel);
* K tiles of 64: both operands by buffer_load_dwordx4 ... lds, 8 rows x 128 B per 1 KiB DMA (whole
  L2 lines), 16 DMAs per wave per tile, into two 64 KiB LDS slots (X rows then W rows, 128-byte
  rows, chunk c of row r at c ^ ((r >> 1) & 7): conflict-free ds_read_b128 for its lane groups);
* three fragment sets in VGPRs: A = v[64:127] (k-half 0 of every tile), B / C = v[128:191] /
  v[192:255] (k-half 1 of even / odd tiles); a tile's fragments are ALL read during the previous
  tile's second phase, so its LDS slot is free from that tile's end and the DMAs two tiles ahead
  get three MFMA phases to land (a two-set schedule freed the slot one phase later and gave them
  one and a half: 5-9 % slower, scripts/exp/gen_w4asm.py);
* per tile t: phase 1 = 64 MFMAs on A (k0 of t) with the 8 W-part DMAs of tile t+2 into slot
  t % 2 (one per 8 MFMAs); vmcnt(8) (this wave's DMAs of tile t+1 landed) + s_barrier; phase 2 =
  64 MFMAs on B|C (k1 of t) with the 32 ds_read_b128 of tile t+1 (k0 -> A, k1 -> the other of
  B|C) one per MFMA over the first 32, then the 8 X-part DMAs of tile t+2 over the second 32
  (away from the reads; W first: 0.3-5 % faster than all 16 in phase 1, X-first split slower on
  gate, scripts/exp/gen_w4asm.py "splitwx"); lgkmcnt(0) + s_barrier.  Every wait counted by hand;
* the last two tiles are peeled: their DMA slots carry the epilogue's reference (yref) tile, half
  h (rows 128 h ..) into slot (K / 64 + h) % 2 with the 16-byte chunk c of row r at c ^ (r & 15),
  so the epilogue reads it from LDS without a load round trip.
The ring slots alternate at run time (an SGPR XOR per tile); the loop body is two tiles (the
k-half-1 set alternates), so K % 128 == 0.
"""
from pathlib import Path

OUT = Path(__file__).resolve().parents[1] / "tensorrt-model-optimizer_amd" / "csrc" / "mtq_awq_w4.inc"
SET_BASE = (64, 128, 192)  # A, B, C
MFMA = {"BF16": "v_mfma_f32_16x16x32_bf16", "F16": "v_mfma_f32_16x16x32_f16"}
# placement (after MFMA #): phase-1 DMAs (the W part) and phase-2 DMAs (the X part) of tile t+2,
# phase-2 reads of tile t+1
P1_DMAS = [8 * k + 1 for k in range(8)]
P2_DMAS = [33 + 4 * k for k in range(8)]
P2_READS = list(range(32))


def xf(s, i):
    return SET_BASE[s] + 4 * i


def wf(s, j):
    return SET_BASE[s] + 32 + 4 * j


def mfma(op, s, i, j):
    a = (i * 8 + j) * 4
    return (f"{op} a[{a}:{a + 3}], v[{wf(s, j)}:{wf(s, j) + 3}], "
            f"v[{xf(s, i)}:{xf(s, i) + 3}], a[{a}:{a + 3}]")


def reads(s, xb, wb):
    """16 ds_read_b128 of one k-half into fragment set s (row block i at 16 rows x 128 B)."""
    out = []
    for i in range(8):
        out.append(f"ds_read_b128 v[{xf(s, i)}:{xf(s, i) + 3}], {xb} offset:{i * 2048}")
        out.append(f"ds_read_b128 v[{wf(s, i)}:{wf(s, i) + 3}], {wb} offset:{i * 2048}")
    return out


def kdmas():
    """16 DMAs of one K tile: X then W, 8 x 1 KiB per wave each; M0 = slot + part + 4 KiB half,
    the 1 KiB block step in the instruction offset (the lane offsets subtract it)."""
    out = []
    for part, (rs, vo) in enumerate((("%[xr]", "xo"), ("%[wr]", "wo"))):
        for u in range(8):
            pre = []
            if u % 4 == 0:
                pre = [f"s_add_u32 m0, %[m0s], {part * 32768 + (u // 4) * 4096}", "s_nop 0"]
            out.append(pre + [f"buffer_load_dwordx4 %[{vo}{u}], {rs}, %[kc] offen offset:{(u % 4) * 1024} lds"])
    return out


def ydmas():
    """16 DMAs of one 128-row half of the yref tile: wave w fills rows 32 w + 2 u + (l >> 5) (512 B
    each); each DMA's scalar offset = the half's base %[ybs] + u rows pairs (any issue order), the
    lane's swizzled chunk in yo(u % 8)."""
    out = []
    for u in range(16):
        out.append([f"s_add_u32 m0, %[m0y], {u * 1024}", f"s_mul_i32 %[yso], %[ys2], {u}",
                    "s_add_u32 %[yso], %[yso], %[ybs]",
                    f"buffer_load_dwordx4 %[yo{u % 8}], %[yr], %[yso] offen lds"])
    return out


def tile(op, k1set, yhalf=None):
    """One K tile: k-half 1 of this tile in set k1set (1 = B, 2 = C), the next tile's in the other."""
    if yhalf is None:
        L = ["s_add_u32 %[m0s], %[m0b], %[sdma]", "s_min_u32 %[kc], %[koff], %[klast]",
             "s_add_u32 %[koff], %[koff], 128"]
        dm = kdmas()
    else:
        L = ["s_add_u32 %[m0y], %[m0yb], %[sdma]",
             "s_mov_b32 %[ybs], %[yrb]" if yhalf == 0 else "s_add_u32 %[ybs], %[yrb], %[yh]"]
        dm = ydmas()
    dm = dm[8:] + dm[:8]  # the W part (or the yref half's second 8 rows pairs) first
    for n in range(64):
        L.append(mfma(op, 0, n // 8, n % 8))
        if n in P1_DMAS:
            L += dm[P1_DMAS.index(n)]
    L += ["s_waitcnt vmcnt(8)", "s_barrier", "s_xor_b32 %[srd], %[sdma], 65536",
          "v_add_u32 v60, %[srd], %[xb0]", "v_add_u32 v61, %[srd], %[wb0]",
          "v_add_u32 v62, %[srd], %[xb1]", "v_add_u32 v63, %[srd], %[wb1]"]
    rd = reads(0, "v60", "v61") + reads(3 - k1set, "v62", "v63")
    for n in range(64):
        L.append(mfma(op, k1set, n // 8, n % 8))
        if n in P2_READS:
            L.append(rd[P2_READS.index(n)])
        if n in P2_DMAS:
            L += dm[8 + P2_DMAS.index(n)]
    L += ["s_waitcnt lgkmcnt(0)", "s_barrier", "s_xor_b32 %[sdma], %[sdma], 65536"]
    return L


def body(op):
    L = ["s_nop 4"]  # SGPR inputs fresh from v_readfirstlane, read by buffer instructions
    L += ["s_mov_b32 %[koff], 0", "s_mov_b32 %[sdma], 0"]
    for t in range(2):
        L += ["s_min_u32 %[kc], %[koff], %[klast]", "s_add_u32 %[koff], %[koff], 128",
              f"s_add_u32 %[m0s], %[m0b], {t * 65536}"]
        for d in kdmas():
            L += d
    # the accumulators zeroed while the first two tiles are in flight
    L += [f"v_accvgpr_write_b32 a{r}, 0" for r in range(256)]
    L += ["s_nop 2", "s_waitcnt vmcnt(16)", "s_barrier"]
    L += reads(0, "%[xb0]", "%[wb0]") + reads(1, "%[xb1]", "%[wb1]")
    L += ["s_waitcnt lgkmcnt(0)", "s_barrier"]  # slot 0 free for tile 2's DMAs
    L += ["s_cmp_eq_u32 %[cnt], 0", "s_cbranch_scc1 L_w4_tail_%="]  # K = 128: the two peeled tiles only
    L.append("L_w4_loop_%=:")
    L += tile(op, 1) + tile(op, 2)
    L += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 L_w4_loop_%="]
    L.append("L_w4_tail_%=:")
    L += tile(op, 1, 0) + tile(op, 2, 1)
    # every DMA landed on every wave before the epilogue reads the yref tile; MFMA results settle
    # before the accumulator reads that follow the statement
    L += ["s_waitcnt vmcnt(0)", "s_waitcnt lgkmcnt(0)", "s_barrier", "s_nop 15", "s_nop 15", "s_nop 15"]
    return L


def text():
    t = "// generated by scripts/gen_awq_w4.py -- do not edit\n"
    for key, op in MFMA.items():
        asm = "".join(f'  "{ln}\\n\\t"\n' for ln in body(op))
        t += f"#define MTQ_W4_BODY_{key} \\\n" + asm.replace("\n", " \\\n") + "\n"
    clob = ", ".join(f'"v{r}"' for r in range(60, 256)) + ",\n  " + ", ".join(f'"a{r}"' for r in range(256))
    t += "#define MTQ_W4_CLOBBERS " + clob.replace("\n", " \\\n") + ', "memory", "scc"\n'
    for i in range(8):  # the 32 accumulators of row block i into float o[32]
        rd = " ".join(f'asm volatile("v_accvgpr_read_b32 %0, a{32 * i + r}" : "=v"(o[{r}]));' for r in range(32))
        t += f"#define MTQ_W4_STRIP_{i}(o) {rd}\n"
    return t


if __name__ == "__main__":
    OUT.write_text(text())
    print(OUT)
