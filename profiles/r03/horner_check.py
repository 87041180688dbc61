"""CPU check of the Horner form of the LSERK4 step (dg_rec.hip, round 3): the stability
polynomial P(z) and the inflow weights g[s][k] from the stage recursion in exact rationals of
the double coefficients, then one step of the oracle's AdvecRHS1D in Horner form against
oracle.advec.lserk4_step on a noisy sine (K = 64, N = 4): max relative difference ~2e-16."""
import sys, numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
from oracle import advec as oa, setup1d
from oracle.setup1d import RK4A, RK4B, RK4C
from fractions import Fraction as F

# symbolic recursion in exact rationals of the double coefficients
A = [F(x) for x in RK4A]; B = [F(x) for x in RK4B]
uc = [F(1)] + [F(0)] * 5; rc = [F(0)] * 6
uf = [[F(0)] * 6 for _ in range(5)]; rf = [[F(0)] * 6 for _ in range(5)]
for s in range(5):
  rc = [A[s] * rc[k] + (uc[k - 1] if k else 0) for k in range(6)]
  rf = [[A[s] * rf[q][k] + (uf[q][k - 1] if k else 0) + (1 if (q == s and k == 0) else 0) for k in range(6)] for q in range(5)]
  uc = [uc[k] + B[s] * rc[k] for k in range(6)]
  uf = [[uf[q][k] + B[s] * rf[q][k] for k in range(6)] for q in range(5)]
beta = [float(x) for x in uc]
g = [[float(x) for x in row] for row in uf]
print("beta", beta, [1, 1, 1/2, 1/6, 1/24])
print("g[s][k] (k=0..4):"); [print(s, row[:5], row[5]) for s, row in enumerate(g)]

N, K = 4, 64
S = setup1d.startup1d(N, np.linspace(0, 1, K + 1))
a = 2 * np.pi
x = S["x"]
rng = np.random.default_rng(0)
u = np.sin(2 * np.pi * x) + 0.1 * rng.standard_normal(x.shape)
dt = oa.bench_dt(S)
t = 0.37
ref = oa.lserk4_step(u, t, dt, a, S)
def Z(v, b):  # dt * rhs(v) with inflow value b
  r, _ = oa.advec_rhs_uin(v, b, a, S)
  return dt * r
uin = [oa.inflow_value(a, t + RK4C[s] * dt, "a") for s in range(5)]
bk = [sum(g[s][k] * uin[s] for s in range(5)) for k in range(5)]
# levels: t4 = b4u + b5 Z_{b4/b5}(u); t3 = b3 u + Z_{b3}(t4); ... u_new = u + Z_{b0}(t1)
tt = beta[4] * u + beta[5] * Z(u, bk[4] / beta[5])
for k in (3, 2, 1):
  tt = beta[k] * u + Z(tt, bk[k])
un = u + Z(tt, bk[0])
print("horner vs lserk max rel", np.abs(un - ref).max() / np.abs(ref).max())
