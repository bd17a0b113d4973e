"""Host-side helpers of the reference's utils.py (problem set-up and error norms).

    weighted_L2, weighted_L1, max_norm, print_norms   utils.py:7-26
    fill_sol_and_RHS_vecs                             utils.py:159-210 (vectorised over the grid)
    manufactured_problem                              the variable-thn manufactured solution of
                                                      solve.py:52-80 / apply.py:40-66
    manufactured_problem_constant                     the constant-thn one (solve.py:60-68: thn = 0.75;
                                                      any constant theta here, BASELINE configs[0])
"""
from __future__ import annotations

import numpy as np

PI = np.pi


def weighted_L2(a, b, w):
    q = a - b
    return np.sqrt((w * q * q).sum())


def weighted_L1(a, b, w):
    return (w * abs(a - b)).sum()


def max_norm(a, b):
    return max(abs(a - b))


def print_norms(u_approx, u_vec, dx, dy, n, show_max=True):
    print(f"The L1_norm for n = {n} is {weighted_L1(u_approx, u_vec, dx * dy)}")
    print(f"The L2_norm for n = {n} is {weighted_L2(u_approx, u_vec, dx * dy)}")
    if show_max:
        print(f"The max_norm for n = {n} is {max_norm(u_approx, u_vec)}")


def _broadcast(f, y, x):
    v = f(y, x)
    return np.broadcast_to(np.asarray(v, dtype=np.float64), np.shape(x)).copy()


def fill_sol_and_RHS_vecs(n, u_n_x_fcn, u_n_y_fcn, u_s_x_fcn, u_s_y_fcn, p_fcn, b_n_x_fcn, b_n_y_fcn,
                          b_s_x_fcn, b_s_y_fcn, b_p_fcn):
    """Solution and RHS vectors [u_n, v_n, u_s, v_s, p] sampled at the MAC locations."""
    dx = 1 / n
    dy = 1 / n
    r, c = np.divmod(np.arange(n * n), n)
    yu, xu = -(r + 0.5) * dy, c * dx           # u faces
    yv, xv = -r * dy, (c + 0.5) * dx           # v faces
    yp, xp = -(r + 0.5) * dy, (c + 0.5) * dx   # cell centres
    u_vec = np.concatenate([_broadcast(u_n_x_fcn, yu, xu), _broadcast(u_n_y_fcn, yv, xv),
                            _broadcast(u_s_x_fcn, yu, xu), _broadcast(u_s_y_fcn, yv, xv),
                            _broadcast(p_fcn, yp, xp)])
    b_vec = np.concatenate([_broadcast(b_n_x_fcn, yu, xu), _broadcast(b_n_y_fcn, yv, xv),
                            _broadcast(b_s_x_fcn, yu, xu), _broadcast(b_s_y_fcn, yv, xv),
                            _broadcast(b_p_fcn, yp, xp)])
    return u_vec, b_vec


def manufactured_problem(n, c=1.0, d=-1.0, xi=1.0, etan=1.0, etas=1.0):
    """(u_vec, b_vec) for thn = 0.25 sin(2 pi x) sin(2 pi y) + 0.5 (solve.py:52-80)."""
    nu = 1.0
    S2 = lambda a: np.sin(2 * PI * a)
    C2 = lambda a: np.cos(2 * PI * a)

    def core(y, x, sign, eta):
        return (sign * 4 * c * nu - sign * 4 * d * (8 * eta * nu * PI * PI + xi)
                + 2 * nu * (c - 16 * d * eta * PI * PI) * S2(x) * S2(y)
                + sign * d * xi * S2(x) * S2(x) * S2(y) * S2(y))

    return fill_sol_and_RHS_vecs(
        n,
        lambda y, x: S2(x) * C2(y), lambda y, x: C2(x) * S2(y),
        lambda y, x: -S2(x) * C2(y), lambda y, x: -C2(x) * S2(y),
        lambda y, x: 0.0,
        lambda y, x: C2(y) * S2(x) * core(y, x, 1.0, etan) / (8 * nu),
        lambda y, x: C2(x) * S2(y) * core(y, x, 1.0, etan) / (8 * nu),
        lambda y, x: C2(y) * S2(x) * core(y, x, -1.0, etas) / (8 * nu),
        lambda y, x: C2(x) * S2(y) * core(y, x, -1.0, etas) / (8 * nu),
        lambda y, x: -PI * np.sin(4 * PI * x) * np.sin(4 * PI * y))


def manufactured_problem_constant(n, c=1.0, d=-1.0, xi=1.0, etan=1.0, etas=1.0, theta=0.75):
    """(u_vec, b_vec) for a constant volume fraction thn = theta (ths = 1 - theta), same solution as the
    variable case (solve.py:52-58).  With constant theta the rows of A reduce to
        b_n = (c theta - 2 d xi theta (1 - theta) - 8 pi^2 d eta_n theta) u_n          (u_s = -u_n)
        b_s = (-c (1 - theta) + 2 d xi theta (1 - theta) + 8 pi^2 d eta_s (1 - theta)) u_n
        b_p = -(2 theta - 1) 4 pi cos(2 pi x) cos(2 pi y)                                 (d_div = -1)
    which at theta = 0.75 are the reference's expressions at solve.py:62-68.  Use with
    MultiphaseBlockPreconditioner.set_theta_tables(theta, theta, theta) (constant tables)."""
    nu = 1.0
    th = float(theta)
    S2 = lambda a: np.sin(2 * PI * a)
    C2 = lambda a: np.cos(2 * PI * a)
    kn = (c * nu * th - 2 * d * xi * th * (1 - th) - 8 * PI * PI * d * etan * nu * th) / nu
    ks = (-c * nu * (1 - th) + 2 * d * xi * th * (1 - th) + 8 * PI * PI * d * etas * nu * (1 - th)) / nu
    return fill_sol_and_RHS_vecs(
        n,
        lambda y, x: S2(x) * C2(y), lambda y, x: C2(x) * S2(y),
        lambda y, x: -S2(x) * C2(y), lambda y, x: -C2(x) * S2(y),
        lambda y, x: 0.0,
        lambda y, x: kn * S2(x) * C2(y), lambda y, x: kn * C2(x) * S2(y),
        lambda y, x: ks * S2(x) * C2(y), lambda y, x: ks * C2(x) * S2(y),
        lambda y, x: -(2 * th - 1) * 4 * PI * C2(x) * C2(y))
