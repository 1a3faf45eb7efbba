# Fit of gsr_expf's degree-6 minimax polynomial (render.hip / oracle/gsr_oracle.cpp): exp(r) ~ 1 + r + c2 r^2 + ... + c6 r^6
# on [-ln2/2, ln2/2], minimising the max relative error (LP on a dense grid).  The exhaustive fp32 check is
# tools/exp_poly_check.c (gcc -O2 -fopenmp -ffp-contract=off tools/exp_poly_check.c -lm; ./a.out c2 c3 c4 c5 c6).
import numpy as np
from scipy.optimize import linprog
h = np.log(2)/2
r = np.linspace(-h, h, 4001)
f = np.exp(r)
# p(r) = 1 + r + sum_{i=2..6} c_i r^i ; minimise max |p - f| / f
S = 1e9
A = np.stack([r**i for i in range(2,7)], 1) / f[:,None] * S
b = (f - 1 - r) / f * S
# variables c2..c6, t ; minimise t s.t. |A c - b| <= t
n = A.shape[1]
c = np.zeros(n+1); c[-1] = 1
Aub = np.vstack([np.hstack([A, -np.ones((len(r),1))]), np.hstack([-A, -np.ones((len(r),1))])])
bub = np.concatenate([b, -b])
res = linprog(c, A_ub=Aub, b_ub=bub, bounds=[(None,None)]*n+[(0,None)], method='highs')
co = res.x[:n]
print("max rel err", res.x[-1]/S, "ulps", res.x[-1]/S/2**-24)
for i,v in enumerate(co): print(f"c{i+2} = {np.float32(v)!r}  ({v:.12e})")
np.save("co.npy", co)
