# Operand-bound check for the carry-free group formulas (corda_amd/csrc/ge25519.hpp):
# every fe_mul(f, g) column sum must stay below 2^64 and 19*g below 2^32.
# max column sums of fe_mul(f, g) for per-limb max bounds F[i], G[j]
T = [2**26 + 2**12 if i % 2 == 0 else 2**25 + 2**18 for i in range(10)]
P2 = [2*(2**26-19)] + [2*(2**25-1) if i % 2 else 2*(2**26-1) for i in range(1,10)]
def col(F, G):
    worst = 0
    for k in range(10):
        s = 0
        for i in range(10):
            j = (k - i) % 10
            a = F[i] * (2 if (i & 1) and (j & 1) else 1)
            b = G[j] * (19 if i + j >= 10 else 1)
            assert a < 2**32 and G[j]*19 < 2**32, (F[i], G[j])
            s += a * b
        worst = max(worst, s)
    return worst
def sc(x, F): return [x * f for f in F]
tight = T
two = sc(2, T)
loose_sub = [t + p for t, p in zip(T, P2)]           # a + 2p - b, a tight
loose_sub2 = [2*t + p for t, p in zip(T, P2)]        # a + 2p - b, a 2x
F5 = [2*t + l for t, l in zip(T, loose_sub)]         # 2C + G'
import math
for name, F, G in [("add X3 f=d-c(2x+2p) g=b-a", loose_sub2, loose_sub), ("add Z3 f=d-c g=d+c", loose_sub2, sc(3, T)),
                   ("dbl X3 F' E'", F5, tight), ("dbl Z3 F' G'", F5, loose_sub), ("dbl Y3 G' H'", loose_sub, two),
                   ("add a: t(Y+2p-X) * YpX(2x)", loose_sub, two)]:
    c = col(F, G)
    print("%-32s max col 2^%.3f  19g max 2^%.3f  f2 max 2^%.3f" % (name, math.log2(c), math.log2(max(G)*19), math.log2(2*max(F))))
