"""Find the operand layout of v_mfma_scale_f32_16x16x128_f8f6f4 from tools/mx_probe output."""
import sys
import numpy as np
import torch

raw = open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/probe/mx_probe.bin", "rb").read()
per = 2048 + 2048 + 256 + 256 + 1024
cases = []
for c in range(4):
    b = raw[c * per:(c + 1) * per]
    a = np.frombuffer(b[:2048], np.uint8).reshape(64, 32)
    bb = np.frombuffer(b[2048:4096], np.uint8).reshape(64, 32)
    sa = np.frombuffer(b[4096:4352], np.int32)
    sb = np.frombuffer(b[4352:4608], np.int32)
    d = np.frombuffer(b[4608:], np.float32).reshape(64, 4)
    cases.append((a, bb, sa, sb, d))

dec = lambda x: torch.from_numpy(x.copy()).view(torch.float8_e4m3fn).float().numpy().astype(np.float64)

# D lane layout: col j = l & 15, row i = 4 (l >> 4) + r
def D_of(d):
    D = np.zeros((16, 16))
    for l in range(64):
        for r in range(4):
            D[4 * (l >> 4) + r, l & 15] = d[l, r]
    return D

layouts = {
    "k=32*(l>>4)+j": lambda l, j: 32 * (l >> 4) + j,
    "halves16": lambda l, j: (16 * (l >> 4) + j) if j < 16 else (64 + 16 * (l >> 4) + j - 16),
    "interleave8": lambda l, j: 8 * (l >> 4) + (j % 8) + 32 * (j // 8),
    "interleave4": lambda l, j: 4 * (l >> 4) + (j % 4) + 16 * (j // 4),
    "interleave16": lambda l, j: 16 * (l >> 4) + (j % 16) + 64 * (j // 16),
}

def full(x, kmap, s=None):
    M = np.zeros((16, 128))
    for l in range(64):
        for j in range(32):
            M[l & 15, kmap(l, j)] = dec(x[l, j:j + 1])[0] * (2.0 ** (s[l] - 127) if s is not None else 1.0)
    return M

a, b, sa, sb, d = cases[0]
D = D_of(d)
for name, km in layouts.items():
    A = full(a, km)
    B = full(b, km)
    ok = np.array_equal(A @ B.T, D)
    print("unit scales", name, ok)

for ci in (1, 2, 3):
    a, b, sa, sb, d = cases[ci]
    D = D_of(d)
    for name, km in layouts.items():
        A = full(a, km, sa)
        B = full(b, km, sb)
        print("case", ci, name, np.array_equal(A @ B.T, D), np.abs(A @ B.T - D).max())

print("--- per-row block exponents (A scales random, case 1) ---")
import itertools
a, b, sa, sb, d = cases[1]
D = D_of(d)
A = np.array([[dec(a[l, j:j+1])[0] for j in range(32)] for l in range(64)])
B = np.array([[dec(b[l, j:j+1])[0] for j in range(32)] for l in range(64)])
for i in range(16):
    # partial sums per lane group q for output (i, jcol): lanes i+16q of A with lanes jcol+16q of B
    P = np.array([[A[i + 16 * q] @ B[jc + 16 * q] for jc in range(16)] for q in range(4)])
    sols = [xs for xs in itertools.product(range(3), repeat=4)
            if np.array_equal(sum(2.0 ** xs[q] * P[q] for q in range(4)), D[i])]
    print(i, "solutions", sols, "sa lanes i+16q:", [int(sa[i + 16 * q] - 127) for q in range(4)],
          "sa lanes 4i..4i+3:", [int(sa[(4 * i + q) % 64] - 127) for q in range(4)])

print("--- per-row block exponents under candidate k-layouts ---")
for name, km in layouts.items():
    Af = full(a, km)
    Bf = full(b, km)
    nsol = 0
    rows = []
    for i in range(16):
        P = [Af[i, 32 * kb:32 * kb + 32] @ Bf[:, 32 * kb:32 * kb + 32].T for kb in range(4)]
        sols = [xs for xs in itertools.product(range(3), repeat=4)
                if np.array_equal(sum(2.0 ** xs[q] * P[q] for q in range(4)), D[i])]
        nsol += len(sols) == 1
        rows.append(sols[0] if len(sols) == 1 else None)
    print(name, "rows solved:", nsol)
    if nsol == 16:
        for i in range(16):
            print(" row", i, rows[i], "sa[i+16q]:", [int(sa[i + 16 * q] - 127) for q in range(4)])

print("--- model: lane l holds k = 16(l>>4)+j (j<16), 64+16(l>>4)+j-16 (j>=16); scale of lane i+16kb = block kb of row i ---")
km = layouts["interleave16"]
for ci in range(4):
    a, b, sa, sb, d = cases[ci]
    Af, Bf = full(a, km), full(b, km)
    ea = np.array([[sa[i + 16 * kb] - 127 for kb in range(4)] for i in range(16)])
    eb = np.array([[sb[i + 16 * kb] - 127 for kb in range(4)] for i in range(16)])
    Af = Af * np.repeat(2.0 ** ea, 32, axis=1)
    Bf = Bf * np.repeat(2.0 ** eb, 32, axis=1)
    print("case", ci, "model matches:", np.array_equal(Af @ Bf.T, D_of(d)))
