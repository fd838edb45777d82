#!/usr/bin/env python3
"""Generate the K loop of the one-wave-per-SIMD AWQ search kernel (scripts/exp/awq_w4asm.hip) as one
inline-asm statement per variant: scripts/exp/w4asm_body.inc.

Schedule (the library's 4-wave 256 x 256 shape at the instruction level):
* 4 waves, a 128 x 128 output block each (2 x 2), 64 16x16 accumulators = a[0:255];
* the K loop runs in HALVES of 32 (256 rows x 64 B per operand = 32 KiB per half); an S-slot LDS
  ring (S x 32 KiB) holds halves h+1 .. h+S-1 landed or in flight while half h is computed;
* both operands by buffer_load_dwordx4 ... lds (8 per wave per half), no register staging;
* fragments double-buffered in VGPRs: set h & 1 holds half h (v[128:191] / v[192:255]: X frags
  i = 0..7, then W frags j = 0..7, 4 VGPRs each);
* step h: vmcnt(8 (S-2)) (own DMAs of half h+1 landed) + lgkmcnt(0) (own reads of half h done) +
  s_barrier; then 64 MFMAs on set h & 1, with the 8 DMAs of half h+S into slot h % S (free: every
  wave's reads of half h finished before the barrier) and the 16 ds_read_b128 of half h+1 into
  the other set interleaved between them (ORDER);
* the ring slots rotate at run time (SGPR slot offsets, two VALU adds per step for the read
  addresses), so the loop body is two steps for any S.
Every wait is counted by hand: the compiler sees one opaque statement.
"""
from pathlib import Path

OUT = Path(__file__).resolve().parent / "w4asm_body.inc"

SET_BASE = (128, 192)
SLOT = 32768
# variant: (slots S, ORDER, SWZ, PROBE); SWZ / S are read by the C++ side from the table written below
# OFS 1: one M0 write per 4 DMAs, the 1 KiB LDS block step in the instruction offset (which also
# moves the global address: the C++ side subtracts it from the lane's voffset)
# CACHE: cache-policy bits of the DMAs ("" / "sc1" / "nt" / "sc0 sc1")
# S = 2: the T64 schedule (body_t64), ORDER G / H
# C++-side fields (kW4Epi / kW4Gm): EPI 1 = probe without the reference-tile loads; GM = row tiles
# per XCD tile unit (the product's 8 x 4 units: GM 8)
# EPI 2: the reference tile prefetched into the LDS ring by the last two K tiles (body_t64y)
# EPI 3: T64B (three fragment sets, two barriers per tile, DMAs two tiles ahead from the tile start)
VARIANTS = [
    (2, "front/splitwx/0/a", 2, 0, 1, "", 3, 8),
    (2, "front/splitwx/0/a", 2, 0, 1, "", 3, -8),
    (2, "front/splitwx/0/a", 2, 0, 1, "", 3, -4),
]
CACHE = ""


def xf(s, i):
    return SET_BASE[s] + 4 * i


def wf(s, j):
    return SET_BASE[s] + 32 + 4 * j


def mfma(s, i, j):
    a = (i * 8 + j) * 4
    return (f"v_mfma_f32_16x16x32_bf16 a[{a}:{a + 3}], v[{wf(s, j)}:{wf(s, j) + 3}], "
            f"v[{xf(s, i)}:{xf(s, i) + 3}], a[{a}:{a + 3}]")


def ds_reads(s, xb, wb):
    """16 ds_read_b128 of one half into fragment set s (xb / wb: the half's read addresses)."""
    out = []
    for i in range(8):
        out.append(f"ds_read_b128 v[{xf(s, i)}:{xf(s, i) + 3}], {xb} offset:{i * 1024}")
        out.append(f"ds_read_b128 v[{wf(s, i)}:{wf(s, i) + 3}], {wb} offset:{i * 1024}")
    return out


def dmas(ofs, slot_sgpr=None, slot_imm=0):
    """8 LDS-DMAs of one half (4 X blocks, then 4 W blocks of 1 KiB per wave); kc holds the half's
    K byte offset; the slot base is %[m0s] (+ slot_imm) -- m0s = m0b + slot offset."""
    out = []
    for part, (rs, vo) in enumerate((("%[xr]", "xo"), ("%[wr]", "wo"))):
        for u in range(4):
            base = "%[m0s]" if slot_sgpr else "%[m0b]"
            if ofs:
                pre = [f"s_add_u32 m0, {base}, {slot_imm + part * 16384}", "s_nop 0"] if u == 0 else []
                out.append(pre + [f"buffer_load_dwordx4 %[{vo}{u}], {rs}, %[kc] offen offset:{u * 1024} {CACHE} lds"])
            else:
                out.append([f"s_add_u32 m0, {base}, {slot_imm + part * 16384 + u * 1024}",
                            "s_nop 0",
                            f"buffer_load_dwordx4 %[{vo}{u}], {rs}, %[kc] offen lds"])
    return out


def k_advance(probe, loop=False):
    if loop and probe == 2:  # probe: the loop re-loads halves 0..3 (L2 hits)
        return ["s_and_b32 %[kc], %[koff], 255", "s_add_u32 %[koff], %[koff], 64"]
    return ["s_min_u32 %[kc], %[koff], %[klast]", "s_add_u32 %[koff], %[koff], 64"]


def placement(order):
    """MFMA index after which each DMA (8) / ds_read (16) is issued."""
    if order == "A":
        return list(range(8)), [8 + 3 * k for k in range(16)]
    if order == "B":
        return [48 + 2 * k for k in range(8)], [3 * k for k in range(16)]
    if order == "C":
        return [8 * k + 4 for k in range(8)], [3 * k for k in range(16)]
    if order == "F":  # hipBLASLt-like: reads one per MFMA from the top, DMAs one per 5 after them
        return [18 + 5 * k for k in range(8)], list(range(16))
    if order == "E":
        return [8 * k + 6 for k in range(8)], [4 * k for k in range(16)]
    raise ValueError(order)


def step(cs, S, order, probe, ofs):
    """One step: compute set cs; read half h+1 (slot %[srd]) into set 1 - cs; DMA half h+S into
    slot %[sdma]; rotate both slot offsets."""
    lines = [f"s_waitcnt vmcnt({8 * (S - 2)})", "s_waitcnt lgkmcnt(0)", "s_barrier",
             "v_add_u32 v120, %[srd], %[xb]", "v_add_u32 v121, %[srd], %[wb]",
             "s_add_u32 %[m0s], %[m0b], %[sdma]"]
    lines += k_advance(probe, True)
    dm = dmas(ofs, slot_sgpr=True)
    rd = ds_reads(1 - cs, "v120", "v121")
    pd, pr = placement(order)
    for n in range(64):
        lines.append(mfma(cs, n // 8, n % 8))
        for k, at in enumerate(pd):
            if at == n:
                lines += dm[k]
        for k, at in enumerate(pr):
            if at == n:
                lines.append(rd[k])
    for r in ("sdma", "srd"):
        lines += [f"s_add_u32 %[{r}], %[{r}], {SLOT}", f"s_cmp_eq_u32 %[{r}], {S * SLOT}",
                  f"s_cselect_b32 %[{r}], 0, %[{r}]"]
    return lines


def prologue(S, probe, ofs):
    lines = ["s_nop 4"]
    lines += [f"v_accvgpr_write_b32 a{r}, 0" for r in range(256)]
    lines += ["s_mov_b32 %[koff], 0", "s_mov_b32 %[sdma], 0", f"s_mov_b32 %[srd], {SLOT}"]
    for q in range(S):
        lines += k_advance(probe)
        for d in dmas(ofs, slot_imm=q * SLOT):
            lines += d
    lines += [f"s_waitcnt vmcnt({8 * (S - 1)})", "s_barrier"]
    lines += ds_reads(0, "%[xb]", "%[wb]")
    return lines


def body(S, order, probe, ofs):
    lines = prologue(S, probe, ofs)
    lines.append("L_w4_loop_%=:")
    lines += step(0, S, order, probe, ofs)
    lines += step(1, S, order, probe, ofs)
    lines += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 L_w4_loop_%="]
    lines += ["s_waitcnt vmcnt(0)", "s_waitcnt lgkmcnt(0)", "s_nop 15", "s_nop 15", "s_nop 15"]
    return lines


# ---- T64 schedule: K tiles of 64 (full 128-byte rows per DMA lane group: 8 rows x 128 B per 1 KiB
# DMA, every L2 line requested once per tile), two 64 KiB slots, one barrier per tile:
#   phase 1: MFMAs of k-half 0 (set 0) + reads of k-half 1 of the same tile into set 1;
#   vmcnt(0) (own DMAs of tile t+1 landed) + lgkmcnt(0) + s_barrier;
#   phase 2: MFMAs of k-half 1 (set 1) + reads of k-half 0 of tile t+1 (other slot) into set 0 +
#   the 16 DMAs of tile t+2 into this tile's slot (every wave's reads of it ended before the barrier).
def dmas64(slot_expr, first):
    """16 DMAs of one K tile: X then W, 8 x 1 KiB per wave each (two M0 bases of 4 KiB per part)."""
    out = []
    for part, (rs, vo) in enumerate((("%[xr]", "xo"), ("%[wr]", "wo"))):
        for u in range(8):
            pre = []
            if u % 4 == 0:
                imm = part * 32768 + (u // 4) * 4096
                pre = [f"s_add_u32 m0, {slot_expr}, {imm}", "s_nop 0"]
            out.append(pre + [f"buffer_load_dwordx4 %[{vo}{u}], {rs}, %[kc] offen offset:{(u % 4) * 1024} {CACHE} lds"])
    return out


def reads64(s, xb, wb):
    out = []
    for i in range(8):
        out.append(f"ds_read_b128 v[{xf(s, i)}:{xf(s, i) + 3}], {xb} offset:{i * 2048}")
        out.append(f"ds_read_b128 v[{wf(s, i)}:{wf(s, i) + 3}], {wb} offset:{i * 2048}")
    return out


def ydmas():
    """16 LDS-DMAs of one 128-row half of the reference (yref) tile into the current slot: wave w
    fills rows 32 w + 2 u + (l >> 5) (512 B each), u = 0..15; each DMA's scalar offset computed
    from the half's base %[ybs] (any issue order), the lane's XOR-swizzled chunk in yo(u % 8)."""
    out = []
    for u in range(16):
        out.append([f"s_add_u32 m0, %[m0y], {u * 1024}", f"s_mul_i32 %[yso], %[ys2], {u}",
                    "s_add_u32 %[yso], %[yso], %[ybs]",
                    f"buffer_load_dwordx4 %[yo{u % 8}], %[yr], %[yso] offen lds"])
    return out


def tile64(order, probe, yhalf=None):
    """One K tile (phase 1, barrier, phase 2); yhalf: the two peeled last tiles, whose phase-2 DMAs
    load the reference tile's half yhalf instead of a (past-the-end) K tile."""
    L = []
    # phase 1
    L += ["s_waitcnt lgkmcnt(0)", "v_add_u32 v120, %[sdma], %[xb1]", "v_add_u32 v121, %[sdma], %[wb1]"]
    rd = reads64(1, "v120", "v121")
    for n in range(64):
        L.append(mfma(0, n // 8, n % 8))
        if n >= 2 and (n - 2) % 3 == 0 and (n - 2) // 3 < 16:
            L.append(rd[(n - 2) // 3])
    kadv = "s_min_u32 %[kc], %[koff], %[klast]" if probe != 2 else "s_mov_b32 %[kc], 0"  # probe 2: L2 hits
    L += ["s_waitcnt vmcnt(0)", "s_waitcnt lgkmcnt(0)", "s_barrier",
          "s_xor_b32 %[srd], %[sdma], 65536", "v_add_u32 v122, %[srd], %[xb0]", "v_add_u32 v123, %[srd], %[wb0]"]
    if yhalf is None:
        L += ["s_add_u32 %[m0s], %[m0b], %[sdma]", kadv, "s_add_u32 %[koff], %[koff], 128"]
        dm = dmas64("%[m0s]", False) if probe != 1 else [[]] * 16  # probe 1: no loads in the loop
    else:
        L += ["s_add_u32 %[m0y], %[m0yb], %[sdma]",
              "s_mov_b32 %[yso], %[yrb]" if yhalf == 0 else "s_add_u32 %[yso], %[yrb], %[yh]"]
        dm = ydmas()
    rd = reads64(0, "v122", "v123")
    pr, pd = PHASE2[order]
    for n in range(64):
        L.append(mfma(1, n // 8, n % 8))
        for k, at in enumerate(pd):
            if at == n:
                L += dm[k]
        for k, at in enumerate(pr):
            if at == n:
                L.append(rd[k])
    L += ["s_xor_b32 %[sdma], %[sdma], 65536"]
    return L


# phase-2 placement: (ds_read after MFMA #, DMA after MFMA #)
PHASE2 = {
    "G": ([2 + 3 * k for k in range(16)], [1 + 4 * k for k in range(16)]),
    "H": ([3 * k for k in range(16)], [16 + 3 * k for k in range(16)]),
    "I": ([2 * k + 1 for k in range(16)], [2 * k for k in range(16)]),
    "J": ([3 * k + 1 for k in range(16)], [3 * k for k in range(16)]),
    "K": ([4 * k + 2 for k in range(16)], [4 * k for k in range(16)]),
}


def body_t64y(order, probe):
    """T64 with the reference tile prefetched into the ring by the last two tiles' DMAs; the loop
    runs K / 64 - 2 tiles (%[cnt], may be 0), the last two are peeled."""
    L = ["s_nop 4"]
    L += [f"v_accvgpr_write_b32 a{r}, 0" for r in range(256)]
    L += ["s_mov_b32 %[koff], 0", "s_mov_b32 %[sdma], 0"]
    for t in range(2):
        L += ["s_min_u32 %[kc], %[koff], %[klast]", "s_add_u32 %[koff], %[koff], 128",
              f"s_add_u32 %[m0s], %[m0b], {t * 65536}"]
        for d in dmas64("%[m0s]", True):
            L += d
    L += ["s_waitcnt vmcnt(16)", "s_barrier"]
    L += reads64(0, "%[xb0]", "%[wb0]")
    L += ["s_cmp_eq_u32 %[cnt], 0", "s_cbranch_scc1 L_w4_tail_%="]
    L.append("L_w4_loop_%=:")
    L += tile64(order, probe)
    L += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 L_w4_loop_%="]
    L.append("L_w4_tail_%=:")
    L += tile64(order, probe, 0)
    L += tile64(order, probe, 1)
    L += ["s_waitcnt vmcnt(0)", "s_waitcnt lgkmcnt(0)", "s_barrier", "s_nop 15", "s_nop 15", "s_nop 15"]
    return L


# ---- T64B: three fragment sets (A = v[64:127] k-half 0, B / C = v[128:191] / v[192:255] k-half 1
# of alternate tiles); a tile's fragments are all read during the previous tile's phase 2, so its
# slot is free at that tile's end barrier and the DMAs two tiles ahead are issued in phase 1:
#   phase 1: MFMAs on A (k0 of t) + the 16 DMAs of tile t+2 into slot t % 2;
#   vmcnt(16) (tile t+1 landed) + s_barrier;
#   phase 2: MFMAs on K1 (k1 of t) + 32 reads of tile t+1 (k0 -> A, k1 -> the other k1 set);
#   lgkmcnt(0) + s_barrier.
def xf3(s, i):
    return (64, 128, 192)[s] + 4 * i


def wf3(s, j):
    return (64, 128, 192)[s] + 32 + 4 * j


def mfma3(s, i, j):
    a = (i * 8 + j) * 4
    return (f"v_mfma_f32_16x16x32_bf16 a[{a}:{a + 3}], v[{wf3(s, j)}:{wf3(s, j) + 3}], "
            f"v[{xf3(s, i)}:{xf3(s, i) + 3}], a[{a}:{a + 3}]")


def reads3(s, xb, wb):
    out = []
    for i in range(8):
        out.append(f"ds_read_b128 v[{xf3(s, i)}:{xf3(s, i) + 3}], {xb} offset:{i * 2048}")
        out.append(f"ds_read_b128 v[{wf3(s, i)}:{wf3(s, i) + 3}], {wb} offset:{i * 2048}")
    return out


B3_READS = "spread"   # "spread": one per 2 MFMAs; "front": one per MFMA over the first 32
B3_DMAS = "spread"    # "spread": one per 4 MFMAs; "front": one per 2 over the first 32
B3_PROBE = 0          # 1: no K-tile DMAs in the loop; 2: they re-load tile 0 (L2 hits)
# "split*": 8 DMAs in phase 1, 8 in phase 2's second half; the order of dm indices (X = 0..7, W = 8..15)
# (each DMA group of 4 must keep its M0 write first: dm[0] / dm[4] / dm[8] / dm[12] carry it)
B3_POS = "a"
RWIN = {"win40": [int(k * 40 / 32) for k in range(32)], "win48": [int(k * 48 / 32) for k in range(32)]}
P1POS = {"f": [8 * k + 1 for k in range(8)], "g": [8 * k + 1 for k in range(8)], "a": [8 * k + 1 for k in range(8)], "b": [2 * k + 1 for k in range(8)], "c": [8 * k + 1 for k in range(8)],
         "d": [8 * k + 5 for k in range(8)], "e": [4 * k + 1 for k in range(8)]}
P2POS = {"f": [41 + 2 * k + (k // 2) for k in range(8)], "g": [49 + 2 * k for k in range(8)], "a": [33 + 4 * k for k in range(8)], "b": [33 + 4 * k for k in range(8)], "c": [32 + 2 * k for k in range(8)],
         "d": [35 + 4 * k for k in range(8)], "e": [33 + 4 * k for k in range(8)]}
SPLIT_ORDER = {"split": list(range(16)),
               "splitwx": list(range(8, 16)) + list(range(8)),
               "splitmix": [0, 1, 2, 3, 8, 9, 10, 11, 4, 5, 6, 7, 12, 13, 14, 15]}


def tile3(k1set, yhalf=None):
    nk1 = 3 - k1set  # the next tile's k-half-1 set (B <-> C)
    L = ["s_add_u32 %[m0s], %[m0b], %[sdma]"] if yhalf is None else \
        ["s_add_u32 %[m0y], %[m0yb], %[sdma]",
         "s_mov_b32 %[ybs], %[yrb]" if yhalf == 0 else "s_add_u32 %[ybs], %[yrb], %[yh]"]
    if yhalf is None:
        L += ["s_min_u32 %[kc], %[koff], %[klast]" if B3_PROBE != 2 else "s_mov_b32 %[kc], 0",
              "s_add_u32 %[koff], %[koff], 128"]
        dm = dmas64("%[m0s]", False) if B3_PROBE != 1 else [[]] * 16
    else:
        dm = ydmas()
    for n in range(64):
        L.append(mfma3(0, n // 8, n % 8))
        if B3_DMAS == "spread" and n % 4 == 1:
            L += dm[n // 4]
        if B3_DMAS == "front" and n < 32 and n % 2 == 0:
            L += dm[n // 2]
        if B3_DMAS.startswith("split") and n in P1POS[B3_POS]:
            L += dm[SPLIT_ORDER[B3_DMAS][P1POS[B3_POS].index(n)]]
    L += ["s_waitcnt vmcnt(16)" if not B3_DMAS.startswith("split") else "s_waitcnt vmcnt(8)", "s_barrier",
          "s_xor_b32 %[srd], %[sdma], 65536",
          "v_add_u32 v60, %[srd], %[xb0]", "v_add_u32 v61, %[srd], %[wb0]",
          "v_add_u32 v62, %[srd], %[xb1]", "v_add_u32 v63, %[srd], %[wb1]"]
    rd = reads3(0, "v60", "v61") + reads3(nk1, "v62", "v63")
    for n in range(64):
        L.append(mfma3(k1set, n // 8, n % 8))
        if B3_READS == "spread" and n % 2 == 0:
            L.append(rd[n // 2])
        if B3_READS == "front" and n < 32:
            L.append(rd[n])
        if B3_READS.startswith("win"):  # a window of >= 32 MFMAs: at most one read per position
            for k, at in enumerate(RWIN[B3_READS]):
                if at == n:
                    L.append(rd[k])
        if B3_DMAS.startswith("split") and n in P2POS[B3_POS]:
            L += dm[SPLIT_ORDER[B3_DMAS][8 + P2POS[B3_POS].index(n)]]
    L += ["s_waitcnt lgkmcnt(0)", "s_barrier", "s_xor_b32 %[sdma], %[sdma], 65536"]
    return L


def body_t64b():
    L = ["s_nop 4"]
    L += [f"v_accvgpr_write_b32 a{r}, 0" for r in range(256)]
    L += ["s_mov_b32 %[koff], 0", "s_mov_b32 %[sdma], 0"]
    for t in range(2):
        L += ["s_min_u32 %[kc], %[koff], %[klast]", "s_add_u32 %[koff], %[koff], 128",
              f"s_add_u32 %[m0s], %[m0b], {t * 65536}"]
        for d in dmas64("%[m0s]", True):
            L += d
    L += ["s_waitcnt vmcnt(16)", "s_barrier"]
    L += reads3(0, "%[xb0]", "%[wb0]") + reads3(1, "%[xb1]", "%[wb1]")
    L += ["s_waitcnt lgkmcnt(0)", "s_barrier"]  # slot 0 free for tile 2's DMAs
    L += ["s_cmp_eq_u32 %[cnt], 0", "s_cbranch_scc1 L_w4_tail_%="]
    L.append("L_w4_loop_%=:")
    L += tile3(1) + tile3(2)
    L += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 L_w4_loop_%="]
    L.append("L_w4_tail_%=:")
    L += tile3(1, 0) + tile3(2, 1)
    L += ["s_waitcnt vmcnt(0)", "s_waitcnt lgkmcnt(0)", "s_barrier", "s_nop 15", "s_nop 15", "s_nop 15"]
    return L


def body_t64(order, probe):
    L = ["s_nop 4"]
    L += [f"v_accvgpr_write_b32 a{r}, 0" for r in range(256)]
    L += ["s_mov_b32 %[koff], 0", "s_mov_b32 %[sdma], 0"]
    for t in range(2):
        L += ["s_min_u32 %[kc], %[koff], %[klast]", "s_add_u32 %[koff], %[koff], 128",
              f"s_add_u32 %[m0s], %[m0b], {t * 65536}"]
        for d in dmas64("%[m0s]", True):
            L += d
    L += ["s_waitcnt vmcnt(16)", "s_barrier"]
    L += reads64(0, "%[xb0]", "%[wb0]")
    L.append("L_w4_loop_%=:")
    # phase 1
    L += ["s_waitcnt lgkmcnt(0)", "v_add_u32 v120, %[sdma], %[xb1]", "v_add_u32 v121, %[sdma], %[wb1]"]
    rd = reads64(1, "v120", "v121")
    for n in range(64):
        L.append(mfma(0, n // 8, n % 8))
        if n >= 2 and (n - 2) % 3 == 0 and (n - 2) // 3 < 16:
            L.append(rd[(n - 2) // 3])
    kadv = "s_min_u32 %[kc], %[koff], %[klast]" if probe != 2 else "s_mov_b32 %[kc], 0"  # probe 2: L2 hits
    L += ["s_waitcnt vmcnt(0)", "s_waitcnt lgkmcnt(0)", "s_barrier",
          "s_xor_b32 %[srd], %[sdma], 65536", "v_add_u32 v122, %[srd], %[xb0]", "v_add_u32 v123, %[srd], %[wb0]",
          "s_add_u32 %[m0s], %[m0b], %[sdma]",
          kadv, "s_add_u32 %[koff], %[koff], 128"]
    rd = reads64(0, "v122", "v123")
    dm = dmas64("%[m0s]", False) if probe != 1 else [[]] * 16  # probe 1: no loads in the loop
    if order == "G":
        pr, pd = [2 + 3 * k for k in range(16)], [1 + 4 * k for k in range(16)]
    else:  # "H": reads first, DMAs after
        pr, pd = [3 * k for k in range(16)], [16 + 3 * k for k in range(16)]
    for n in range(64):
        L.append(mfma(1, n // 8, n % 8))
        for k, at in enumerate(pd):
            if at == n:
                L += dm[k]
        for k, at in enumerate(pr):
            if at == n:
                L.append(rd[k])
    L += ["s_xor_b32 %[sdma], %[sdma], 65536",
          "s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 L_w4_loop_%="]
    L += ["s_waitcnt vmcnt(0)", "s_waitcnt lgkmcnt(0)", "s_nop 15", "s_nop 15", "s_nop 15"]
    return L


def strips():
    """W4ASM_STRIP_i(o): the 32 accumulators of row block i (a[32 i .. 32 i + 31]) into float o[32]."""
    out = []
    for i in range(8):
        rd = " ".join(f'asm volatile("v_accvgpr_read_b32 %0, a{32 * i + r}" : "=v"(o[{r}]));' for r in range(32))
        out.append(f"#define W4ASM_STRIP_{i}(o) {rd}\n")
    return "".join(out)


def main():
    text = "// generated by scripts/exp/gen_w4asm.py -- do not edit\n"
    global CACHE
    for v, (S, order, swz, probe, ofs, CACHE, _epi, _gm) in enumerate(VARIANTS):
        if S == 2 and _epi == 3:
            global B3_READS, B3_DMAS, B3_PROBE
            global B3_POS
            B3_READS, B3_DMAS, pr = order.split("/")[:3]
            B3_POS = order.split("/")[3] if order.count("/") >= 3 else "a"
            B3_PROBE = int(pr)
            lines = body_t64b()
        elif S == 2:
            lines = body_t64y(order, probe) if _epi == 2 else body_t64(order, probe)
        else:
            lines = body(S, order, probe, ofs)
        asm = "".join(f'  "{ln}\\n\\t"\n' for ln in lines)
        name = f"W4ASM_BODY_{v}" if _epi < 2 else f"W4ASM_BODY_Y_{v}"
        text += f"#define {name} \\\n" + asm.replace("\n", " \\\n") + "\n"
    text += f"#define W4ASM_NVAR {len(VARIANTS)}\n"
    text += "constexpr int kW4Slots[] = {" + ", ".join(str(v[0]) for v in VARIANTS) + "};\n"
    text += "constexpr int kW4Swz[] = {" + ", ".join(str(v[2]) for v in VARIANTS) + "};\n"
    text += "constexpr int kW4Ofs[] = {" + ", ".join(str(v[4]) for v in VARIANTS) + "};\n"
    text += "constexpr int kW4Epi[] = {" + ", ".join(str(v[6]) for v in VARIANTS) + "};\n"
    text += "constexpr int kW4Gm[] = {" + ", ".join(str(v[7]) for v in VARIANTS) + "};\n"
    clob = ", ".join(f'"v{r}"' for r in range(60, 256)) + ",\n  " + ", ".join(f'"a{r}"' for r in range(256))
    text += "#define W4ASM_CLOBBERS " + clob.replace("\n", " \\\n") + ', "memory", "scc"\n'
    text += strips()
    OUT.write_text(text)


if __name__ == "__main__":
    main()
