"""Can the low-nibble UTF-8 table lose its bit-3 blend?

The "byte before" low-nibble table of csrc/utf8_device.hpp (t2, 16 entries)
costs per dword: sel_lo = x & 7, the bit-3 mask m_lo (a perm of x << 4 and
x << 12, the shifts shared by a dword pair), two perms and a blend; then t12 =
t1 & t2.  A cheaper form would look t2 up by ONE v_perm_b32 over a selector
computed from the nibble in one or two instructions, using the perm's own
special selectors (8-11: the sign bits of table bytes 1/3/5/7 replicated,
12: 0x00, 13 and up: 0xFF), with t12 = bitop3(t1, t2raw, K) absorbing a bit
polarity.  The t2 bits that matter: 2 (overlong 3, nibble 0), 3 (too large,
nibble >= 4), 4 (surrogate, nibble D), 5 (overlong 2, nibble <= 1), 7 (overlong
4 / too large 1000, nibble 0 or >= 5); bits 0, 1 and 6 are 1 for every nibble.

This searches the selector families below for one that reproduces the table
(the classes {0}, {1}, {2,3}, {4}, {D}, rest); each prints its count of
solutions, and every count is 0: the blend stays ("The UTF-8
tables, round 6").
  - any v_bitop3_b32 of the byte with two constants (upper nibble zeroed)
  - that, plus a constant added (bytes do not carry into each other)
  - the nibble plus a constant, then any per-bit function of the sum's 5 bits
  - an XOR by a constant then any monotone map (v_lerp_u8, adds, saturation)
usage: python3 tools/utf8_selector_search.py
"""
from __future__ import annotations

import itertools

DESIRED = [0xE7, 0x63, 0x43, 0x43, 0x4B] + [0xCB] * 8 + [0xDB, 0xCB, 0xCB]  # t2 by nibble
VAR = 0xBC  # bits 2, 3, 4, 5, 7


def f3(tt, a, b, x):
    return (tt >> ((x << 2) | (a << 1) | b)) & 1


def check(s, mode, K=0):
    """Is there an 8-byte table for selector map s (nibble -> selector byte)?
    mode 'xor': t12 = t1 & (t2raw ^ K), every bit exact; 'id' / 'not': the
    varying bits taken as they are / inverted, bits 0, 1, 6 passed from t1."""
    if mode == "xor":
        req = [(d ^ K, 0xFF) for d in DESIRED]
    elif mode == "id":
        req = [(d & VAR, VAR) for d in DESIRED]
    else:
        req = [(~d & VAR, VAR) for d in DESIRED]
    groups = {}
    for n, sv in enumerate(s):
        v, m = req[n]
        if sv in groups:
            v0, m0 = groups[sv]
            if (v ^ v0) & m & m0:
                return None
            groups[sv] = ((v0 & m0) | (v & m), m | m0)
        else:
            groups[sv] = (v, m)
    table = {}
    for sv, (v, m) in groups.items():
        if sv == 12 and v & m:
            return None
        if sv >= 13 and (v & m) != m:
            return None
        if sv < 8:
            table[sv] = (v, m)
    for sv, (v, m) in groups.items():
        if 8 <= sv <= 11:
            if v & m not in (0, m):
                return None
            want = 1 if v & m else 0
            pos = 2 * (sv - 8) + 1
            tv, tm = table.get(pos, (0, 0))
            if tm & 0x80 and (tv >> 7) & 1 != want:
                return None
            table[pos] = (tv | (0x80 if want else 0), tm | 0x80)
    return table


def bitwise_maps():
    maps = set()
    for tt in range(256):
        if not any(f3(tt, a, b, 0) == 0 and f3(tt, a, b, 1) == 0 for a in (0, 1) for b in (0, 1)):
            continue  # the byte's upper nibble could not be zeroed
        for A in range(16):
            for B in range(16):
                maps.add(tuple(sum(f3(tt, (A >> k) & 1, (B >> k) & 1, (n >> k) & 1) << k for k in range(4))
                               for n in range(16)))
    return maps


def main():
    maps = bitwise_maps()
    one = sum(1 for s in maps for mode in ("id", "not") if check(s, mode) is not None)
    one += sum(1 for s in maps for K in range(256) if check(s, "xor", K) is not None)
    print("one bitop3 of the byte:", one)
    two = sum(1 for s in maps for c in range(14) for mode in ("id", "not")
              if check([x + c for x in s], mode) is not None)
    print("bitop3 then add:", two)
    add_first = 0
    for c in range(17):
        for fns in itertools.product(range(4), repeat=5):
            s = []
            for n in range(16):
                y, o = n + c, 0
                for k, fn in enumerate(fns):
                    yb = (y >> k) & 1
                    o |= (0 if fn == 0 else 1 if fn == 1 else yb if fn == 2 else 1 - yb) << k
                s.append(o)
            add_first += sum(1 for mode in ("id", "not") if check(s, mode) is not None)
    print("add then per-bit map:", add_first)
    cls = [0, 1, 2, 2, 3] + [4] * 8 + [5, 4, 4]
    mono = 0
    for X in range(16):
        seq = [cls[n] for n in sorted(range(16), key=lambda n: n ^ X)]
        runs = [c for i, c in enumerate(seq) if i == 0 or c != seq[i - 1]]
        mono += len(runs) == len(set(runs))  # every class one interval of n ^ X
    print("xor then monotone:", mono)


if __name__ == "__main__":
    main()
