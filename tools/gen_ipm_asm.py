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
    parts.append("}  // namespace osc\n")
    with open(OUT, "w") as f:
        f.write("\n".join(parts))
    print(OUT)


if __name__ == "__main__":
    main()
