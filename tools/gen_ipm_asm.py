"""Generate operational-space-control_amd/csrc/osc_ipm_asm.hpp: the interior point's triangular
solves and its Hr y product as single inline-asm statements (round 6).

Why: a wavefront alone on its SIMD (the interior point at 4,096 Go2 envs) pays ~4.5 clocks for
every instruction it issues, s_nop included (tools/mb/mb_issue.hip), and hipcc pads the boundary
between two dependent inline-asm statements with an s_nop (its conservative forwarding-hazard rule
for asm producers on gfx950).  The per-step asm statements of ldl_fwd_rows / ldl_bwd_rows /
dot_rows (osc_ipm.hpp) cost an s_nop per step that way; one statement per solve, scheduled by
hand, needs none: each step's lane-mask compare is issued one step early (the mask's one wait
state) and each DPP read of a value written by the previous step's FMA sits two instructions
after it (the selects are the wait states).  Same instructions on the same values in the same
order per accumulator as the C++ forms: bitwise the same results.

    python tools/gen_ipm_asm.py        (rewrites the header)"""
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "operational-space-control_amd", "csrc", "osc_ipm_asm.hpp")
ROW = 16
DPP = " row_mask:0xf bank_mask:0xf"


def fmac(dst, src, m, k):
    return f"v_fmac_f64_dpp {reg(dst)}, {reg(src)}, %[{m}] row_newbcast:{k}{DPP}"


# a0, a1, z0, z1 live in fixed VGPR pairs (register constraints): the selects need their halves,
# which an operand of the asm cannot name
PIN = {"a0": 0, "a1": 2, "z0": 4, "z1": 6}


def reg(name):
    return f"v[{PIN[name]}:{PIN[name] + 1}]" if name in PIN else f"%[{name}]"


def sel(dst, set_):
    # dst = vcc ? set : dst, 64-bit as two halves
    d, s_ = PIN[dst], PIN[set_]
    return [f"v_cndmask_b32 v{d}, v{d}, v{s_}, vcc",
            f"v_cndmask_b32 v{d + 1}, v{d + 1}, v{s_ + 1}, vcc"]


def cmp(k):
    return f"v_cmp_eq_u32 vcc, {k}, %[l]"


def fwd(n):
    ins = ["s_nop 1", cmp(0)]
    for k in range(n):
        kl = k % ROW
        last = k == n - 1
        if k < ROW:
            ins += sel("z0", "a0")
            if k < ROW - 1:
                ins.append(fmac("a1", "a0", f"c1_{k}", kl))
                ins.append(cmp((k + 1) % ROW))
                ins.append(fmac("a0", "a0", f"c0_{k}", kl))
            else:   # k = 15: no slot-0 update; the compare goes before the FMA (its wait state)
                ins.append(cmp((k + 1) % ROW))
                ins.append(fmac("a1", "a0", f"c1_{k}", kl))
        else:
            ins += sel("z1", "a1")
            if not last:
                ins.append(cmp((k + 1) % ROW))
            ins.append(fmac("a1", "a1", f"c1_{k}", kl))
    uses = [f"c0_{k}" for k in range(ROW - 1)] + [f"c1_{k}" for k in range(n)]
    return ins, uses


def bwd(n):
    ins = ["s_nop 1", cmp((n - 1) % ROW)]
    for k in range(n - 1, -1, -1):
        kl = k % ROW
        if k >= ROW:
            ins += sel("z1", "a1")
            if k > ROW:
                ins.append(fmac("a0", "a1", f"c0_{k}", kl))
                ins.append(cmp((k - 1) % ROW))
                ins.append(fmac("a1", "a1", f"c1_{k}", kl))
            else:   # k = 16: no slot-1 update
                ins.append(cmp((k - 1) % ROW))
                ins.append(fmac("a0", "a1", f"c0_{k}", kl))
        else:
            ins += sel("z0", "a0")
            if k >= 1:
                ins.append(cmp((k - 1) % ROW))
                ins.append(fmac("a0", "a0", f"c0_{k}", kl))
    uses = [f"c0_{k}" for k in range(1, n)] + [f"c1_{k}" for k in range(ROW + 1, n)]
    return ins, uses


def dot(n):
    ins = ["s_nop 1"]
    for i in range(n):
        src = "x0" if i < ROW else "x1"
        acc = ("a", "b") if i % 2 == 0 else ("a2", "b2")
        ins.append(fmac(acc[0], src, f"ma_{i}", i % ROW))
        ins.append(fmac(acc[1], src, f"mb_{i}", i % ROW))
    return ins


def asm_text(ins):
    return "\n".join(f'      "{t}\\n\\t"' for t in ins)


def emit_solve(name, n, ins, uses, doc):
    ins_ops = ", ".join(f'[{u}] "v"({u[:2]}[{u[3:]}])' for u in uses) + ', [l] "v"(l)'
    return f"""// {doc}
template <>
__device__ __forceinline__ void {name}<{n}>(const double (&c0)[{n}], const double (&c1)[{n}],
                                           double& a0, double& a1, double& z0, double& z1, int l) {{
  asm volatile(
{asm_text(ins)}
      : [a0] "+{{v[0:1]}}"(a0), [a1] "+{{v[2:3]}}"(a1), [z0] "+{{v[4:5]}}"(z0), [z1] "+{{v[6:7]}}"(z1)
      : {ins_ops}
      : "vcc");
}}
"""


def emit_dot(n):
    ops = ", ".join([f'[ma_{i}] "v"(ma[{i}])' for i in range(n)] +
                    [f'[mb_{i}] "v"(mb[{i}])' for i in range(n)])
    return f"""template <>
__device__ __forceinline__ void dot_rows_asm<{n}>(double& a, double& b, double& a2, double& b2,
                                                double x0, double x1, const double (&ma)[{n}],
                                                const double (&mb)[{n}]) {{
  asm volatile(
{asm_text(dot(n))}
      : [a] "+v"(a), [b] "+v"(b), [a2] "+v"(a2), [b2] "+v"(b2)
      : [x0] "v"(x0), [x1] "v"(x1), {ops});
}}
"""


def main():
    with open(OUT, "w") as f:
        f.write(render())
    print(OUT)


def render():
    parts = [f"""// osc_ipm_asm.hpp -- GENERATED by tools/gen_ipm_asm.py (do not edit): the interior point's
// triangular solves and Hr y product, one inline-asm statement each (see the generator's notes).
// Included by osc_ipm.hpp; N = the reduced QP's size (24: unitree_go2, 32: walter_sr).
#pragma once

namespace osc {{

// forward  z = L^-1 r over the factor ldl_rows leaves (osc_ipm.hpp ldl_fwd_rows): a0 / a1 in,
// z0 / z1 (zero on entry) out
template <int N>
__device__ __forceinline__ void ldl_fwd_asm(const double (&c0)[N], const double (&c1)[N],
                                            double& a0, double& a1, double& z0, double& z1, int l);
// backward (osc_ipm.hpp ldl_bwd_rows, before the 1 / D scaling): a0 / a1 in, z0 / z1 out
template <int N>
__device__ __forceinline__ void ldl_bwd_asm(const double (&c0)[N], const double (&c1)[N],
                                            double& a0, double& a1, double& z0, double& z1, int l);
// LDL^T in place (osc_ipm.hpp ldl_rows<N, true>): 1 / D_k to LDS at byte address addr + 8 k
template <int N>
__device__ __forceinline__ void ldl_asm(double (&c0)[N], double (&c1)[N], double thr0, double thr1,
                                        int l, unsigned addr, double du);
// a += sum_i bcast(x_i) ma[i] over the even i, a2 over the odd ones (b, b2 with mb)
template <int N>
__device__ __forceinline__ void dot_rows_asm(double& a, double& b, double& a2, double& b2,
                                             double x0, double x1, const double (&ma)[N],
                                             const double (&mb)[N]);
"""]
    for n in (24, 32):
        ins, uses = fwd(n)
        parts.append(emit_solve("ldl_fwd_asm", n, ins, uses, f"N = {n}: forward solve"))
        ins, uses = bwd(n)
        parts.append(emit_solve("ldl_bwd_asm", n, ins, uses, f"N = {n}: backward solve"))
        parts.append(emit_dot(n))
        parts.append(emit_ldl(n))
    parts.append("}  // namespace osc\n")
    return "\n".join(parts)



# ----------------------------------------------------------------------------------------------
# LDL^T of the Newton matrix (osc_ipm.hpp ldl_rows, GUARD form) as one asm statement, scheduled
# by a small list scheduler: pivot k+1's preparation (test, broadcast, reciprocal, scaling, the
# next multipliers) is interleaved with pivot k's trailing FMAs so that every wait state the
# hardware needs is an FMA instead of an s_nop.  Temporaries whose 32-bit halves the selects
# need live in clobbered VGPRs (an asm operand cannot name a pair's halves).
SCR = {"B": 244, "G": 246, "D": 248, "R": 250, "S0": 252, "S1": 254}   # B: 1e128
BIG_LO, BIG_HI = "0xf9301d32", "0x5a827748"   # 1e128


def r64(name):
    if name in SCR:
        return f"v[{SCR[name]}:{SCR[name] + 1}]"
    return f"%[{name}]"


class Ins:
    def __init__(self, text, w=(), r=(), dpp=(), trans=False, wvcc=False, rvcc=False):
        self.text, self.w, self.r, self.dpp = text, set(w), set(r), set(dpp)
        self.trans, self.wvcc, self.rvcc = trans, wvcc, rvcc


def ldl_prep(k, n):
    s, kl = k // ROW, k % ROW
    own = f"c{s}_{k}"
    thr = f"thr{s}"
    G, D, R = SCR["G"], SCR["D"], SCR["R"]
    S = f"S{k % 2}"
    Sr = SCR[S]
    # slot 0: the pivot gets the torque rows' diagonal term du (osc_ipm.hpp ldl_rows)
    first = (Ins(f"v_add_f64 v[{G}:{G + 1}], {r64(own)}, %[du]", w=["G"], r=[own, "du"]) if s == 0
             else Ins(f"v_mov_b64 v[{G}:{G + 1}], {r64(own)}", w=["G"], r=[own]))
    p = [first,
         Ins(f"v_cmp_gt_f64 vcc, v[{G}:{G + 1}], %[{thr}]", r=["G", thr], wvcc=True),
         Ins(f"v_cndmask_b32 v{G}, v{SCR['B']}, v{G}, vcc", w=["G"], r=["G", "B"], rvcc=True),
         Ins(f"v_cndmask_b32 v{G + 1}, v{SCR['B'] + 1}, v{G + 1}, vcc", w=["G"], r=["G", "B"], rvcc=True),
         Ins(f"v_mov_b64_dpp v[{D}:{D + 1}], v[{G}:{G + 1}] row_newbcast:{kl}{DPP}", w=["D"], dpp=["G"]),
         Ins(f"v_rcp_f64 v[{R}:{R + 1}], v[{D}:{D + 1}]", w=["R"], r=["D"], trans=True),
         Ins(f"v_fma_f64 v[{G}:{G + 1}], -v[{D}:{D + 1}], v[{R}:{R + 1}], 1.0", w=["G"], r=["D", "R"]),
         Ins(f"v_fma_f64 v[{D}:{D + 1}], v[{R}:{R + 1}], v[{G}:{G + 1}], v[{R}:{R + 1}]", w=["D"], r=["R", "G"]),
         Ins(f"ds_write_b64 %[addr], v[{D}:{D + 1}] offset:{8 * k}", r=["addr", "D"])]
    # scaling: the column the next multipliers come from goes through S (its halves), the other
    # in place; t1 = c1[k] itself while k < 16
    if k < ROW - 1:          # t0 = keep_gt<k>(c0[k]), t1 = c1[k]
        p += [Ins(f"v_mul_f64 v[{Sr}:{Sr + 1}], -{r64('c0_' + str(k))}, v[{D}:{D + 1}]", w=[S], r=[f"c0_{k}", "D"]),
              Ins(f"v_mul_f64 {r64('c1_' + str(k))}, -{r64('c1_' + str(k))}, v[{D}:{D + 1}]", w=[f"c1_{k}"], r=[f"c1_{k}", "D"]),
              Ins(f"v_mov_b64 {r64('c0_' + str(k))}, v[{Sr}:{Sr + 1}]", w=[f"c0_{k}"], r=[S]),
              Ins(f"v_cmp_lt_u32 vcc, {kl}, %[l]", r=["l"], wvcc=True),
              Ins(f"v_cndmask_b32 v{Sr}, 0, v{Sr}, vcc", w=[S], r=[S], rvcc=True),
              Ins(f"v_cndmask_b32 v{Sr + 1}, 0, v{Sr + 1}, vcc", w=[S], r=[S], rvcc=True)]
    elif k < ROW:            # k = 15: no slot-0 updates follow; t1 = c1[15]
        p += [Ins(f"v_mul_f64 {r64('c0_' + str(k))}, -{r64('c0_' + str(k))}, v[{D}:{D + 1}]", w=[f"c0_{k}"], r=[f"c0_{k}", "D"]),
              Ins(f"v_mul_f64 {r64('c1_' + str(k))}, -{r64('c1_' + str(k))}, v[{D}:{D + 1}]", w=[f"c1_{k}"], r=[f"c1_{k}", "D"])]
    else:                    # t1 = keep_gt<k - 16>(c1[k])
        p += [Ins(f"v_mul_f64 {r64('c0_' + str(k))}, -{r64('c0_' + str(k))}, v[{D}:{D + 1}]", w=[f"c0_{k}"], r=[f"c0_{k}", "D"]),
              Ins(f"v_mul_f64 v[{Sr}:{Sr + 1}], -{r64('c1_' + str(k))}, v[{D}:{D + 1}]", w=[S], r=[f"c1_{k}", "D"]),
              Ins(f"v_mov_b64 {r64('c1_' + str(k))}, v[{Sr}:{Sr + 1}]", w=[f"c1_{k}"], r=[S]),
              Ins(f"v_cmp_lt_u32 vcc, {kl}, %[l]", r=["l"], wvcc=True),
              Ins(f"v_cndmask_b32 v{Sr}, 0, v{Sr}, vcc", w=[S], r=[S], rvcc=True),
              Ins(f"v_cndmask_b32 v{Sr + 1}, 0, v{Sr + 1}, vcc", w=[S], r=[S], rvcc=True)]
    return p


def ldl_mults(k):
    """register names of step k's multipliers (t0, t1)"""
    s = k // ROW
    t0 = f"S{k % 2}" if k < ROW - 1 else None
    t1 = f"c1_{k}" if k < ROW else f"S{k % 2}"
    return t0, t1


def ldl_upd(k, i):
    s, kl = k // ROW, k % ROW
    t0, t1 = ldl_mults(k)
    if s == 0:
        rows = [Ins(f"v_fmac_f64_dpp {r64('c1_' + str(i))}, {r64('c0_' + str(i))}, {r64(t1)} row_newbcast:{kl}{DPP}",
                    w=[f"c1_{i}"], r=[f"c1_{i}", t1], dpp=[f"c0_{i}"])]
        if k < ROW - 1:
            rows.append(Ins(f"v_fmac_f64_dpp {r64('c0_' + str(i))}, {r64('c0_' + str(i))}, {r64(t0)} row_newbcast:{kl}{DPP}",
                            w=[f"c0_{i}"], r=[f"c0_{i}", t0], dpp=[f"c0_{i}"]))
        return rows
    return [Ins(f"v_fmac_f64_dpp {r64('c1_' + str(i))}, {r64('c1_' + str(i))}, {r64(t1)} row_newbcast:{kl}{DPP}",
                w=[f"c1_{i}"], r=[f"c1_{i}", t1], dpp=[f"c1_{i}"])]


class Sched:
    def __init__(self):
        self.out = []          # emitted texts
        self.hist = []         # (Ins or None for nop slots) per issue slot

    def need(self, ins):
        """wait states still missing before ins can issue"""
        miss = 0
        for back, prev in enumerate(reversed(self.hist)):   # back = slots between prev and now
            if prev is None:
                continue
            if ins.dpp & prev.w and back < 2:
                miss = max(miss, 2 - back)
            if prev.trans and (ins.r | ins.dpp) & prev.w and back < 1:
                miss = max(miss, 1 - back)
            if prev.wvcc and ins.rvcc and back < 2:
                miss = max(miss, 2 - back)
            if back >= 2:
                break
        return miss

    def emit(self, ins):
        m = self.need(ins)
        if m:
            self.out.append(f"s_nop {m - 1}")
            self.hist += [None] * m
        self.out.append(ins.text)
        self.hist.append(ins)


def ldl(n):
    sc = Sched()
    B = SCR["B"]   # 1e128 (a VOP2 select cannot take a literal and VCC: one constant-bus read)
    sc.emit(Ins(f"v_mov_b32 v{B}, {BIG_LO}", w=["B"]))
    sc.emit(Ins(f"v_mov_b32 v{B + 1}, {BIG_HI}", w=["B"]))
    for ins in ldl_prep(0, n):
        sc.emit(ins)
    for k in range(n):
        if k + 1 < n:
            for ins in ldl_upd(k, k + 1):
                sc.emit(ins)
            chain = ldl_prep(k + 1, n)
            fill = [ins for i in range(k + 2, n) for ins in ldl_upd(k, i)]
            while chain:
                if sc.need(chain[0]) == 0 or not fill:
                    sc.emit(chain.pop(0))
                else:
                    sc.emit(fill.pop(0))
            for ins in fill:
                sc.emit(ins)
    uses = [f"c0_{i}" for i in range(n)] + [f"c1_{i}" for i in range(n)]
    return sc.out, uses


def emit_ldl(n):
    ins, uses = ldl(n)
    outs = ", ".join(f'[{u}] "+v"({u[:2]}[{u[3:]}])' for u in uses)
    clob = ", ".join(f'"v{r}"' for base in SCR.values() for r in (base, base + 1))
    return f"""// N = {n}: LDL^T, {sum(1 for t in ins if not t.startswith("s_nop"))} instructions, {sum(int(t.split()[1]) + 1 for t in ins if t.startswith("s_nop"))} wait slots
template <>
__device__ __forceinline__ void ldl_asm<{n}>(double (&c0)[{n}], double (&c1)[{n}], double thr0,
                                           double thr1, int l, unsigned addr, double du) {{
  asm volatile(
{asm_text(ins)}
      : {outs}
      : [thr0] "v"(thr0), [thr1] "v"(thr1), [l] "v"(l), [addr] "v"(addr), [du] "v"(du)
      : "vcc", "memory", {clob});
}}
"""


if __name__ == "__main__":
    main()
