"""Diagnostic: numpy model of the device LM (MINPACK lmder control flow on
normal equations) driven by the oracle's residual/Jacobian.  Used to tell
conditioning effects (normal equations vs QR) apart from device bugs."""
import sys

import numpy as np
import scipy.linalg as sla

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from oracle import refcpu as R  # noqa: E402


REFINE = 0


def lm_ne(fun, jac, x0, m, ftol=1e-6, xtol=1e-6, gtol=1e-6, maxfev=1000, factor=100.0):
    n = len(x0)
    x = np.array(x0, float)
    f = fun(x); nfev = 1; trace = [np.linalg.norm(f)]
    fnorm = trace[0]; par = 0.0; it = 1; njev = 0; info = 0
    diag = np.zeros(n); delta = xnorm = 0
    while True:
        J = jac(x, f); njev += 1
        A = J.T @ J; g = J.T @ f; acn = np.sqrt(np.diag(A))
        if it == 1:
            diag = np.where(acn == 0, 1.0, acn)
            xnorm = np.linalg.norm(diag * x); delta = factor * xnorm or factor
        gnorm = np.max(np.where(acn != 0, np.abs(g / fnorm) / np.where(acn == 0, 1, acn), 0)) if fnorm else 0
        if gnorm <= gtol:
            info = 4; break
        diag = np.maximum(diag, acn)
        while True:
            def solve(lam):
                Al = A + lam * np.diag(diag ** 2)
                c = sla.cho_factor(Al, lower=True)
                xs = sla.cho_solve(c, g)
                for _ in range(REFINE):
                    # corrected semi-normal equations (Bjorck): residual from J, not A
                    r = J.T @ (f - J @ xs) - lam * diag ** 2 * xs
                    xs = xs + sla.cho_solve(c, r)
                return xs, c
            xs, c0 = solve(0.0)
            dx = np.linalg.norm(diag * xs); fp = dx - delta
            if fp <= 0.1 * delta:
                par = 0.0
            else:
                v = diag * (diag * xs / dx)
                t = np.sqrt(v @ sla.cho_solve(c0, v)); parl = fp / delta / t / t
                gn = np.linalg.norm(g / diag); paru = gn / delta
                if paru == 0: paru = np.finfo(float).tiny / min(delta, 0.1)
                par = min(max(par, parl), paru)
                if par == 0: par = gn / dx
                k = 0
                while True:
                    k += 1
                    if par == 0: par = max(np.finfo(float).tiny, 0.001 * paru)
                    xs, c = solve(par); dx = np.linalg.norm(diag * xs)
                    tmp = fp; fp = dx - delta
                    if abs(fp) <= 0.1 * delta or (parl == 0 and fp <= tmp and tmp < 0) or k == 10:
                        break
                    v = diag * (diag * xs / dx)
                    t = np.sqrt(v @ sla.cho_solve(c, v)); parc = fp / delta / t / t
                    if fp > 0: parl = max(parl, par)
                    if fp < 0: paru = min(paru, par)
                    par = max(parl, par + parc)
            p = -xs; x2 = x + p; pnorm = np.linalg.norm(diag * p)
            print("ne  trial: delta=%.17g par=%.17g pnorm=%.17g" % (delta, par, pnorm), file=sys.stderr)
            if it == 1: delta = min(delta, pnorm)
            f2 = fun(x2); nfev += 1; fn1 = np.linalg.norm(f2); trace.append(fn1)
            actred = 1 - (fn1 / fnorm) ** 2 if 0.1 * fn1 < fnorm else -1.0
            t1 = np.linalg.norm(J @ p) / fnorm; t2 = np.sqrt(par) * pnorm / fnorm
            prered = t1 * t1 + t2 * t2 / 0.5; dirder = -(t1 * t1 + t2 * t2)
            ratio = actred / prered if prered != 0 else 0.0
            if ratio <= 0.25:
                temp = 0.5 if actred >= 0 else 0.5 * dirder / (dirder + 0.5 * actred)
                if 0.1 * fn1 >= fnorm or temp < 0.1: temp = 0.1
                delta = temp * min(delta, pnorm / 0.1); par /= temp
            elif par == 0 or ratio >= 0.75:
                delta = pnorm / 0.5; par *= 0.5
            if ratio >= 1e-4:
                x = x2; f = f2; xnorm = np.linalg.norm(diag * x); fnorm = fn1; it += 1
            if abs(actred) <= ftol and prered <= ftol and 0.5 * ratio <= 1: info = 1
            if delta <= xtol * xnorm: info = 2
            if abs(actred) <= ftol and prered <= ftol and 0.5 * ratio <= 1 and info == 2: info = 3
            if info: return x, info, nfev, njev, trace
            if nfev >= maxfev: info = 5
            if info: return x, info, nfev, njev, trace
            if ratio >= 1e-4: break
    return x, info, nfev, njev, trace


if __name__ == "__main__":
    from mayamatchmovesolver_amd import synthetic as S
    idx = int(sys.argv[1]); frames = int(sys.argv[2]); scale = float(sys.argv[3])
    REFINE = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    p = S.make_config(idx, frames=frames, scale=scale); o = S.config_options(p)
    fun = lambda x: R.measure(p, o, x)[0]
    def jac(x, f):
        return R.jacobian(p, o, x)[1]
    R.lib().ref_set_debug(1)
    xr, fr, eur, edr, rr, trr = R.solve(p, o)
    xn, info, nfev, njev, tr = lm_ne(fun, jac, p.x0, p.num_residuals, maxfev=o.iter_max)
    print("ref:", rr.reason_number, rr.iterations, rr.outer_iterations)
    print("ne :", info, nfev, njev)
    k = min(len(tr), len(trr))
    print(np.array(tr[:k]) / np.array(trr[:k]) - 1)
    print("x rel", np.max(np.abs(xn - xr) / np.maximum(np.abs(xr), 1e-3)))
