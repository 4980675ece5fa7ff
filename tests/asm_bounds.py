"""Interval (bound) interpreter for the generated gfx950 assembly products (test infrastructure).

tests/asm_sim.py runs the generators' instruction lists on concrete values; this module runs the
same lists on INTERVALS: every register, LDS word and scalar constant holds [lo, hi], every
instruction maps intervals to the interval of its result, and every v_mad_u64_u32 /
v_mad_i64_i32 / v_lshl_add_u64 is checked to stay inside [0, 2^64) for EVERY operand in the
input intervals -- a proof of the column bounds the generators claim (worst case over all inputs,
not over the inputs a concrete test happens to draw), used to decide which accumulator slots need
the mid-product reduction.  Addresses, loop counters and offsets must be concrete (lo == hi).
Only the instructions the one-lane generator (tools/gen_nadic_asm.py) emits are modelled.
"""

import re

M32 = (1 << 32) - 1
M64 = (1 << 64) - 1
_PAIR = re.compile(r"^([vs])\[(\d+):(\d+)\]$")
_ONE = re.compile(r"^([vs])(\d+)$")


def _parse(ln):
    op, _, rest = ln.partition(" ")
    ops = [t.strip() for t in rest.split(",")] if rest else []
    if "_dpp" in op:  # DPP controls (quad_perm / wave shifts, masks, bound_ctrl) follow the last operand
        ops = [t.split()[0] if " " in t and not t.startswith("0x") else t for t in ops]
        ops = [t for t in ops if not t.startswith(("quad_perm", "row_mask", "bank_mask", "bound_ctrl", "wave_"))]
    off = 0
    if ops and "offset:" in ops[-1]:
        last, _, o = ops[-1].partition("offset:")
        off = int(o, 0)
        ops[-1] = last.strip()
    return op, ops, off


class Overflow(AssertionError):
    pass


class BoundLane:
    """One lane; values are (lo, hi) pairs.  `peaks` records, per destination register of every
    64-bit accumulate, the largest hi seen (by instruction index: tag)."""

    def __init__(self, args, lds=None, smem=None, glb=None):
        self.r, self.p = {}, {}
        self.args = {k: (v, v) if isinstance(v, int) else v for k, v in args.items()}
        self.lds = lds if lds is not None else {}
        self.smem = smem if smem is not None else {}
        self.glb = glb if glb is not None else {}
        self.scc = 0
        self.max_mad = 0

    # -- operands -----------------------------------------------------------------------------
    def get(self, tok):
        m = re.fullmatch(r"%\[(\w+)\]", tok)
        if m:
            return self.args[m.group(1)]
        if tok in ("vcc", "m0"):
            return self.r.get(tok, (0, 0))
        m = _PAIR.match(tok)
        if m:
            k, lo, hi = m.group(1), int(m.group(2)), int(m.group(3))
            assert hi == lo + 1
            key = f"{k}{lo}"
            if key in self.p:
                return self.p[key]
            a, b = self.r.get(key, (0, 0)), self.r.get(f"{k}{hi}", (0, 0))
            return (a[0] + (b[0] << 32), a[1] + (b[1] << 32))
        if _ONE.match(tok):
            if tok not in self.r:
                raise KeyError(f"read of unwritten register {tok}")
            return self.r[tok]
        v = int(tok, 0)
        return (v, v)

    def _kill_pairs(self, reg):
        k, n = reg[0], int(reg[1:])
        self.p.pop(f"{k}{n}", None)
        self.p.pop(f"{k}{n - 1}", None)

    def put(self, tok, iv):
        lo, hi = iv
        assert 0 <= lo <= hi, (tok, iv)
        if tok in ("vcc", "m0"):
            self.r[tok] = (lo & M32, hi & M32) if hi <= M32 else (0, M32)
            return
        m = _PAIR.match(tok)
        if m:
            k, a = m.group(1), int(m.group(2))
            assert hi <= M64, (tok, iv)
            self._kill_pairs(f"{k}{a}")
            self._kill_pairs(f"{k}{a + 1}")
            self.p[f"{k}{a}"] = (lo, hi)
            self.r[f"{k}{a}"] = (lo, hi) if hi <= M32 else (0, M32)
            self.r[f"{k}{a + 1}"] = (lo >> 32, hi >> 32)
            return
        assert _ONE.match(tok), tok
        assert hi <= M32, (tok, iv)
        self._kill_pairs(tok)
        self.r[tok] = (lo, hi)

    @staticmethod
    def _conc(iv, what):
        assert iv[0] == iv[1], f"{what} must be concrete, got {iv}"
        return iv[0]

    # -- one instruction ------------------------------------------------------------------------
    def step(self, op, ops, off):
        g = self.get
        if op in ("s_waitcnt", "s_nop"):
            return
        if op.startswith("s_load_dword"):
            n = {"s_load_dwordx2": 2, "s_load_dwordx4": 4, "s_load_dwordx8": 8, "s_load_dwordx16": 16}[op]
            m = _PAIR.match(ops[0])
            base = self._conc(g(ops[1]), "s_load base") + int(ops[2], 0)
            for i in range(n):
                self.r[f"s{int(m.group(2)) + i}"] = self.smem[base + 4 * i]
            return
        if op == "global_load_dword":
            addr = self._conc(g(ops[2]), "global base") + self._conc(g(ops[1]), "global offset") + off
            self.put(ops[0], self.glb[addr])
            return
        if op == "ds_read_b32":
            addr = self._conc(g(ops[1]), "LDS address") + off
            self.put(ops[0], self.lds[addr])
            return
        if op == "ds_read_b64":
            addr = self._conc(g(ops[1]), "LDS address") + off
            a, b = self.lds[addr], self.lds[addr + 4]
            self.put(ops[0], (a[0] + (b[0] << 32), a[1] + (b[1] << 32)))
            return
        if op == "ds_write_b32":
            addr = self._conc(g(ops[0]), "LDS address") + off
            self.lds[addr] = g(ops[1])
            return
        if op in ("v_mov_b32", "s_mov_b32"):
            self.put(ops[0], g(ops[1]))
            return
        if op in ("v_add_u32", "s_add_u32"):
            a, b = g(ops[1]), g(ops[2])
            if op == "v_add_u32" and a[1] + b[1] > M32:
                raise Overflow(f"v_add_u32 may wrap: {ops} {a} {b}")
            self.put(ops[0], (a[0] + b[0], a[1] + b[1]))
            return
        if op == "v_sub_u32":
            a, b = g(ops[1]), g(ops[2])
            lo, hi = a[0] - b[1], a[1] - b[0]
            if lo < 0:
                raise Overflow(f"v_sub_u32 may go negative: {ops} {a} {b}")
            self.put(ops[0], (lo, hi))
            return
        if op == "v_and_b32":
            a, b = g(ops[1]), g(ops[2])
            if a[0] != a[1] and b[0] != b[1]:  # a lane-dependent mask (%[mq]): below both
                self.put(ops[0], (0, min(a[1], b[1])))
                return
            mask, val = (a, b) if a[0] == a[1] and (b[0] != b[1] or a[0] & (a[0] + 1) == 0) else (b, a)
            mk = mask[0]
            assert mask[0] == mask[1]
            if val[1] <= mk and (mk & (mk + 1)) == 0:  # a low-bits mask covering the value
                self.put(ops[0], val)
            else:
                self.put(ops[0], (0, min(val[1], mk)))
            return
        if op == "v_mul_lo_u32":
            self.put(ops[0], (0, M32))
            return
        if op == "v_lshlrev_b32":
            k = self._conc(g(ops[1]), "shift")
            a = g(ops[2])
            self.put(ops[0], (a[0] << k, a[1] << k))
            return
        if op == "v_mad_u64_u32":
            a, b, c = g(ops[2]), g(ops[3]), g(ops[4])
            assert a[1] <= M32 and b[1] <= M32
            lo, hi = a[0] * b[0] + c[0], a[1] * b[1] + c[1]
            if hi > M64:
                raise Overflow(f"v_mad_u64_u32 may overflow: {ops} a={a} b={b} c={c}")
            self.max_mad = max(self.max_mad, hi)
            self.put(ops[0], (lo, hi))
            self.put(ops[1], (0, 0))
            return
        if op == "v_mad_i64_i32":  # only as  d = c - a  (a * -1 + c)
            assert ops[3] == "-1", ops
            a, c = g(ops[2]), g(ops[4])
            lo, hi = c[0] - a[1], c[1] - a[0]
            if lo < 0:
                raise Overflow(f"v_mad_i64_i32 may go negative: {ops} a={a} c={c}")
            self.put(ops[0], (lo, hi))
            self.put(ops[1], (0, 0))
            return
        if op == "v_lshrrev_b64":
            k = self._conc(g(ops[1]), "shift")
            a = g(ops[2])
            self.put(ops[0], (a[0] >> k, a[1] >> k))
            return
        if op == "v_lshl_add_u64":
            a, k, c = g(ops[1]), self._conc(g(ops[2]), "shift"), g(ops[3])
            lo, hi = (a[0] << k) + c[0], (a[1] << k) + c[1]
            if hi > M64:
                raise Overflow(f"v_lshl_add_u64 may overflow: {ops}")
            self.put(ops[0], (lo, hi))
            return
        # ---- the lane-group engines (tools/gen_quad_asm.py), bounded on ONE abstract lane whose
        # intervals are the hull over the group's lanes: a cross-lane read (DPP, ds_bpermute) reads the
        # same register's hull; a DPP read past the wave's ends (bound_ctrl) reads 0, inside the hull ----
        if op in ("v_and_b32_dpp", "v_mov_b32_dpp"):
            src = g(ops[1])
            if op == "v_mov_b32_dpp":
                self.put(ops[0], (0, src[1]))
            else:
                mk = g(ops[2])
                self._conc(mk, "DPP mask")
                self.put(ops[0], (0, min(src[1], mk[0])))
            return
        if op == "v_add_u32_dpp":  # the triple's DPP broadcast (gen_quad_asm.dpp_bcast): a sum over a group's
            # lanes of a digit masked with %[mq], nonzero in the group's lane 0 only -- so the sum is one lane's
            # value and stays inside the larger hull (asm_sim checks the values lane by lane)
            a, b = g(ops[1]), g(ops[2])
            self.put(ops[0], (0, max(a[1], b[1])))
            return
        if op == "ds_bpermute_b32":
            src = g(ops[2])
            self.put(ops[0], (0, src[1]))
            return
        if op in ("v_add_co_u32", "v_addc_co_u32"):
            a, b = g(ops[2]), g(ops[3])
            c = g(ops[4]) if op == "v_addc_co_u32" else (0, 0)
            lo, hi = a[0] + b[0] + c[0], a[1] + b[1] + c[1]
            self.put(ops[0], (lo, hi) if hi <= M32 else (0, M32))
            self.put(ops[1], (lo >> 32, hi >> 32))
            return
        if op == "v_alignbit_b32":
            hi_, lo_, k = g(ops[1]), g(ops[2]), self._conc(g(ops[3]), "shift")
            a, b = ((hi_[0] << 32) + lo_[0]) >> k, ((hi_[1] << 32) + lo_[1]) >> k
            self.put(ops[0], (a, b) if b <= M32 else (0, M32))
            return
        if op == "s_movrels_b32":
            m = _ONE.match(ops[1])
            self.put(ops[0], self.r[f"s{int(m.group(2)) + self._conc(self.r['m0'], 'm0')}"])
            return
        if op == "s_cmp_lg_u32":
            self.scc = int(self._conc(g(ops[0]), "s_cmp") != self._conc(g(ops[1]), "s_cmp"))
            return
        raise NotImplementedError(op)

    def run(self, lines, max_steps=2_000_000):
        prog, labels = [], {}
        for ln in lines:
            ln = ln.strip()
            if ln.endswith(":"):
                labels[ln[:-1]] = len(prog)
                continue
            prog.append(_parse(ln))
        pc = steps = 0
        while pc < len(prog):
            steps += 1
            assert steps < max_steps
            op, ops, off = prog[pc]
            pc += 1
            if op == "s_cbranch_scc1":
                if self.scc:
                    pc = labels[ops[0].rstrip("bf")]
                continue
            self.step(op, ops, off)
        return self
