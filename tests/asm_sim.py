"""Lockstep interpreter for the generated gfx950 assembly products (test infrastructure).

Runs the instruction list a generator (tools/gen_nadic_asm.py: one lane per ciphertext,
tools/gen_quad_asm.py: four or three) emits for ONE lane (`Lane.run`) or for lanes in
lockstep (`Wave.run`: DPP quad_perm / wave_shl:1 / wave_shr:1 and ds_bpermute_b32 read another
lane's register -- wave shifts with bound_ctrl read 0 past either end --, scalar state is
per-lane but identical), with LDS / global memory / the scalar constants block as shared
dictionaries, so the register plan, offsets, loop control, cross-lane steps and arithmetic
of the assembly are checked on the CPU against Python integers before they run on a GPU.
Every v_mad_u64_u32 is checked not to overflow 64 bits (the column bounds the generators
claim).  Only the instructions the generators use are implemented; anything else raises.
"""

import re

M32 = (1 << 32) - 1
M64 = (1 << 64) - 1
_PAIR = re.compile(r"^([vs])\[(\d+):(\d+)\]$")
_ONE = re.compile(r"^([vs])(\d+)$")
_QPERM = re.compile(r"quad_perm:\[(\d),(\d),(\d),(\d)\]")
_WSHIFT = re.compile(r"wave_(shl|shr):1")


def _size(ln):
    """Encoded size in bytes (gfx9): VOP3 / DS / FLAT / SMEM 8, VOP2 / SOP 4, +4 for a
    literal, DPP +4."""
    op, _, rest = ln.partition(" ")
    ops = [t.strip() for t in rest.split(",")] if rest else []
    if op.startswith(("v_mad", "v_mul_lo", "v_lshrrev_b64", "v_lshl_add", "v_alignbit", "ds_", "global_",
                      "s_load")):
        return 8
    if "_dpp" in op:
        return 8
    lit = any(re.fullmatch(r"0x[0-9a-f]+|\d+", t) and int(t, 0) > 64 for t in ops[1:]) or any(
        t.startswith(".L") for t in ops)
    return 4 + (4 if lit else 0)


def _parse(ln):
    """(op, operands, offset, cross-lane source: quad_perm tuple, +1 (wave_shl:1: lane i reads
    lane i + 1), -1 (wave_shr:1) or None)"""
    perm = None
    m = _QPERM.search(ln)
    if m:
        perm = tuple(int(m.group(i)) for i in range(1, 5))
        ln = ln[:m.start()].rstrip()
    m = _WSHIFT.search(ln)
    if m:
        if "bound_ctrl:0" not in ln:
            raise NotImplementedError("wave shifts are only modelled with bound_ctrl:0 (0 past the ends)")
        perm = 1 if m.group(1) == "shl" else -1
        ln = ln[:m.start()].rstrip()
    ln = re.sub(r"\s+(row_mask|bank_mask|bound_ctrl):\S+", "", ln)
    op, _, rest = ln.partition(" ")
    ops = [t.strip() for t in rest.split(",")] if rest else []
    off = 0
    if ops and "offset:" in ops[-1]:
        last, _, o = ops[-1].partition("offset:")
        off = int(o, 0)
        ops[-1] = last.strip()
    return op, ops, off, perm


class Lane:
    def __init__(self, args, lds=None, glb=None, smem=None):
        self.r = {}
        self.args = args            # placeholder name -> int value (addresses, scalars)
        self.lds = lds if lds is not None else {}
        self.glb = glb if glb is not None else {}
        self.smem = smem if smem is not None else {}
        self.scc = 0
        self.vcc = 0

    # -- operands -------------------------------------------------------------------------
    def _sub(self, tok):
        m = re.fullmatch(r"%\[(\w+)\]", tok)
        return ("arg", m.group(1)) if m else None

    def get(self, tok):
        a = self._sub(tok)
        if a:
            return self.args[a[1]]
        if tok == "vcc":
            return self.vcc
        if tok == "m0":
            return self.r.get("m0", 0)
        m = _PAIR.match(tok)
        if m:
            k, lo, hi = m.group(1), int(m.group(2)), int(m.group(3))
            v = 0
            for i in range(hi, lo - 1, -1):
                v = (v << 32) | self.r.get(f"{k}{i}", 0)
            return v
        m = _ONE.match(tok)
        if m:
            if tok not in self.r:
                raise KeyError(f"read of unwritten register {tok}")
            return self.r[tok]
        return int(tok, 0)

    def put(self, tok, val):
        if tok == "m0":
            self.r["m0"] = val & M32
            return
        if tok == "vcc":
            self.vcc = val
            return
        m = _PAIR.match(tok)
        if m:
            k, lo, hi = m.group(1), int(m.group(2)), int(m.group(3))
            for i in range(lo, hi + 1):
                self.r[f"{k}{i}"] = val & M32
                val >>= 32
            return
        if _ONE.match(tok):
            self.r[tok] = val & M32
            return
        raise ValueError(f"bad destination {tok}")

    def _expr(self, tok):
        """operand or a label difference '.La - .Lb' (byte distance, as the assembler resolves it)"""
        m = re.fullmatch(r"(\.[\w%=]+)\s*-\s*(\.[\w%=]+)", tok)
        if m:
            return self._byte_labels[m.group(1)] - self._byte_labels[m.group(2)]
        return self.get(tok)

    # -- one instruction --------------------------------------------------------------------
    def step(self, op, ops, off, pc, ctx):
        """Executes one instruction for this lane; returns the next pc."""
        if op in ("s_waitcnt", "s_nop"):
            return pc
        if op.startswith("s_load_dword"):
            n = {"s_load_dwordx2": 2, "s_load_dwordx4": 4, "s_load_dwordx8": 8, "s_load_dwordx16": 16}[op]
            m = _PAIR.match(ops[0])
            base = self.get(ops[1]) + int(ops[2], 0)
            for i in range(n):
                self.r[f"s{int(m.group(2)) + i}"] = self.smem[base + 4 * i]
        elif op == "global_load_dword":
            addr = self.get(ops[2]) + self.get(ops[1]) + off
            self.put(ops[0], self.glb[addr])
        elif op == "global_load_dwordx4":  # dst v[a:a+3], 64-bit VGPR address, "off" (no SGPR base)
            assert ops[2] == "off"
            addr = self.get(ops[1]) + off
            assert addr % 16 == 0, f"global_load_dwordx4 address {addr}"
            self.put(ops[0], sum(self.glb[addr + 4 * i] << (32 * i) for i in range(4)))
        elif op == "ds_read_b32":
            addr = self.get(ops[1]) + off
            self.put(ops[0], self.lds.get(addr, 0))
        elif op == "ds_read_b64":
            addr = self.get(ops[1]) + off
            assert addr % 8 == 0, f"ds_read_b64 address {addr}"
            self.put(ops[0], self.lds.get(addr, 0) | (self.lds.get(addr + 4, 0) << 32))
        elif op == "ds_write_b32":
            addr = self.get(ops[0]) + off
            self.lds[addr] = self.get(ops[1])
        elif op in ("v_mov_b32", "s_mov_b32"):
            self.put(ops[0], self.get(ops[1]))
        elif op == "v_add_u32":
            self.put(ops[0], self.get(ops[1]) + self.get(ops[2]))
        elif op == "v_add_co_u32":
            v = self.get(ops[2]) + self.get(ops[3])
            self.put(ops[0], v)
            self.put(ops[1], v >> 32)
        elif op == "v_addc_co_u32":
            v = self.get(ops[2]) + self.get(ops[3]) + (self.get(ops[4]) & 1)
            self.put(ops[0], v)
            self.put(ops[1], v >> 32)
        elif op == "s_add_u32":
            v = self.get(ops[1]) + self._expr(ops[2])
            self.scc = v >> 32
            self.put(ops[0], v)
        elif op == "v_sub_u32":
            self.put(ops[0], self.get(ops[1]) - self.get(ops[2]))
        elif op == "v_and_b32":
            self.put(ops[0], self.get(ops[1]) & self.get(ops[2]))
        elif op == "v_mul_lo_u32":
            self.put(ops[0], self.get(ops[1]) * self.get(ops[2]))
        elif op == "v_lshlrev_b32":
            self.put(ops[0], self.get(ops[2]) << self.get(ops[1]))
        elif op == "v_bfe_u32":
            self.put(ops[0], (self.get(ops[1]) >> self.get(ops[2])) & ((1 << self.get(ops[3])) - 1))
        elif op == "v_alignbit_b32":
            self.put(ops[0], (((self.get(ops[1]) << 32) | self.get(ops[2])) >> (self.get(ops[3]) & 31)) & M32)
        elif op == "v_mad_u64_u32":
            a, b = self.get(ops[2]), self.get(ops[3])
            assert a <= M32 and b <= M32
            v = a * b + self.get(ops[4])
            assert v <= M64, f"v_mad_u64_u32 overflow: {ops}"
            self.put(ops[0], v)
            self.put(ops[1], 0)  # the carry-out (vcc or a rotated SGPR pair): 0, as asserted above
        elif op == "v_mad_i64_i32":  # signed: the engines use it as  column - q  (q * -1 + column)
            def s32(x):
                return x - (1 << 32) if x >> 31 else x
            a, b = s32(self.get(ops[2]) & M32), s32(self.get(ops[3]) & M32)
            v = a * b + self.get(ops[4])
            assert 0 <= v <= M64, f"v_mad_i64_i32 out of [0, 2^64): {ops}"
            self.put(ops[0], v)
            self.put(ops[1], 0)
        elif op == "v_lshrrev_b64":
            self.put(ops[0], self.get(ops[2]) >> self.get(ops[1]))
        elif op == "v_lshl_add_u64":
            v = (self.get(ops[1]) << self.get(ops[2])) + self.get(ops[3])
            assert v <= M64, f"v_lshl_add_u64 overflow: {ops}"
            self.put(ops[0], v)
        elif op == "s_getpc_b64":
            self.put(ops[0], ctx["baddr"][pc] if pc < len(ctx["baddr"]) else ctx["pos"])
        elif op == "s_setpc_b64":
            target = self.get(ops[0])
            if target not in ctx["at"]:
                raise RuntimeError(f"jump into the middle of an instruction: {target}")
            return ctx["at"][target]
        elif op == "s_addc_u32":
            v = self.get(ops[1]) + self.get(ops[2]) + self.scc
            self.scc = v >> 32
            self.put(ops[0], v)
        elif op == "s_lshl_b32":
            self.put(ops[0], self.get(ops[1]) << self.get(ops[2]))
        elif op == "s_movrels_b32":
            m = _ONE.match(ops[1])
            self.put(ops[0], self.r[f"s{int(m.group(2)) + self.r['m0']}"])
        elif op == "v_movrels_b32":
            m = _ONE.match(ops[1])
            self.put(ops[0], self.r[f"v{int(m.group(2)) + self.r['m0']}"])
        elif op == "s_cmp_lg_u32":
            self.scc = int(self.get(ops[0]) != self.get(ops[1]))
        elif op == "s_cbranch_scc1":
            if self.scc:
                return ctx["labels"][ops[0].rstrip("bf")]
        else:
            raise NotImplementedError(op)
        return pc

    def run(self, lines, max_steps=10_000_000):
        return Wave([self]).run(lines, max_steps)


class Wave:
    """Lanes executing one instruction stream in lockstep (a quad of a wave)."""

    def __init__(self, lanes):
        self.lanes = lanes

    def run(self, lines, max_steps=10_000_000):
        prog, labels, baddr, byte_labels = [], {}, [], {}
        pos = 0
        for ln in lines:
            ln = ln.strip()
            if ln.endswith(":"):
                labels[ln[:-1]] = len(prog)
                byte_labels[ln[:-1]] = pos
                continue
            prog.append(_parse(ln))
            baddr.append(pos)
            pos += _size(ln)
        ctx = {"labels": labels, "baddr": baddr, "pos": pos, "at": {a: i for i, a in enumerate(baddr)}}
        for ln in self.lanes:
            ln._byte_labels = byte_labels
        pc, steps, counts = 0, 0, {}
        n = len(self.lanes)
        while pc < len(prog):
            steps += 1
            if steps > max_steps:
                raise RuntimeError("step cap")
            op, ops, off, perm = prog[pc]
            pc += 1
            counts[op] = counts.get(op, 0) + 1
            if op == "ds_bpermute_b32":  # dst <- data of lane addr / 4 (every lane reads, then writes)
                vals = []
                for lane in self.lanes:
                    a = lane.get(ops[1]) + off
                    assert a % 4 == 0 and 0 <= a // 4 < n, f"ds_bpermute address {a}"
                    vals.append(a)
                vals = [self.lanes[a // 4].get(ops[2]) for a in vals]
                for i, lane in enumerate(self.lanes):
                    lane.put(ops[0], vals[i])
                continue
            if perm is not None:
                # every lane reads src0 from its source lane (within its quad, or the next /
                # previous lane of the wave) before any lane writes; a VOP2 takes src1 from its own lane
                if isinstance(perm, tuple):
                    src = [self.lanes[(i & ~3) + perm[i & 3]].get(ops[1]) if (i & ~3) + perm[i & 3] < n else 0
                           for i in range(n)]
                else:
                    src = [self.lanes[i + perm].get(ops[1]) if 0 <= i + perm < n else 0 for i in range(n)]
                if op == "v_mov_b32_dpp":
                    vals = src
                elif op == "v_and_b32_dpp":
                    vals = [src[i] & lane.get(ops[2]) for i, lane in enumerate(self.lanes)]
                elif op == "v_add_u32_dpp":
                    vals = [(src[i] + lane.get(ops[2])) & M32 for i, lane in enumerate(self.lanes)]
                else:
                    raise NotImplementedError(op)
                for i, lane in enumerate(self.lanes):
                    lane.put(ops[0], vals[i])
                continue
            nxt = [lane.step(op, ops, off, pc, ctx) for lane in self.lanes]
            if len(set(nxt)) != 1:
                raise RuntimeError(f"lanes diverged at {op} {ops}")
            pc = nxt[0]
        return counts
