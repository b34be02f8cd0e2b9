# Host design check (numpy, fp64; not product code — the kernel is csrc/lane_kernel.h, SEG
# instantiations): the horizon-partitioned Riccati of one PDAS pass (fixed active set) against
# the sequential Riccati of the same equality-constrained LQ problem.
#
# Problem (one QP, recentred, x_0 = 0; mpc.cpp:208-306 with the gap rows inactive): stages
# i = 0..N-1, x_{i+1} = A x_i + B u_i + C (model.cpp:42-55), cost sum_i 1/2|x_i - r_i|_Q^2 +
# 1/2|u_i - ud|_R^2 + 1/2|x_N - r_{N-1}|_Q^2 (mpc.cpp:228); a fixed input sits on its bound.
#
# Segments j = 0..S-1 cover stages [s_j, e_j). Each segment runs the Riccati recursion backward
# over its own stages with the terminal value V_e(x_e) = lam_j' x_e (lam_j: the multiplier of the
# coupling x_e^(j) = x_s^(j+1); the last segment keeps the true terminal cost), and alongside it
# the affine map x_e = Phi x_s + psi + Gam lam_j of the closed loop:
#   Phi_i = Phi_{i+1} (A + B K_i),  W = Phi_{i+1} B,  F_i = -S^-1 W' (lam-gain of u_i),
#   Gam_i = Gam_{i+1} + W F_i,      psi_i = Phi_{i+1}(B k_i + C) + psi_{i+1}.
# At the segment start V_s(x) = 1/2 x'P x + (a + Phi' lam)' x + ...; the coupling conditions
#   x_s^(j+1) = Phi_j x_s^(j) + psi_j + Gam_j lam_j,   lam_{j-1} = P_j x_s^(j) + a_j + Phi_j' lam_j
# are an LQ two-point boundary problem over the S segment ends, solved by a Riccati recursion
# over the segments (lam_{j-1} = M_j x_s^(j) + m_j). Then each segment rolls forward from its
# x_s with u_i = K_i x_i + k_i + F_i lam_j.
import numpy as np


def model(rng, N, heading=True):
    dt = 0.01
    v = rng.uniform(0.5, 4.5)
    d = rng.uniform(-0.4, 0.4)
    th = rng.uniform(-np.pi, np.pi) if not heading else 0.0
    L = 0.3302
    sn, cs = np.sin(th), np.cos(th)
    A = np.eye(3)
    A[0, 2] = -v * sn * dt
    A[1, 2] = v * cs * dt
    B = np.zeros((3, 2))
    B[0, 0] = cs * dt
    B[1, 0] = sn * dt
    B[2, 0] = np.tan(d) * dt / L
    B[2, 1] = v / np.cos(d) ** 2 * dt / L
    C = np.array([0.0, 0.0, -d * v / np.cos(d) ** 2 * dt / L])
    return A, B, C


def masked_inv(H, fixed):
    f0, f1 = not fixed[0], not fixed[1]
    M00 = H[0, 0] if f0 else 1.0
    M11 = H[1, 1] if f1 else 1.0
    M01 = H[0, 1] if (f0 and f1) else 0.0
    det = M00 * M11 - M01 * M01
    I = np.zeros((2, 2))
    I[0, 0] = M11 / det if f0 else 0.0
    I[1, 1] = M00 / det if f1 else 0.0
    I[0, 1] = I[1, 0] = -M01 / det if (f0 and f1) else 0.0
    return I


def stage(P, p, A, B, C, Q, R, ud, r_i, fixed, bval):
    """One masked Riccati step: returns K, k, P_i, p_i, Sinv (masked)."""
    g = P @ C + p
    Huu = R + B.T @ P @ B
    X = B.T @ P @ A
    Y = Q + A.T @ P @ A
    h = -R @ ud + B.T @ g
    hx = -Q @ r_i + A.T @ g
    I = masked_inv(Huu, fixed)
    bA = np.array([bval[0] if fixed[0] else 0.0, bval[1] if fixed[1] else 0.0])
    K = -I @ X
    w = h + Huu @ bA
    k = bA - I @ w
    return K, k, Y + X.T @ K, hx + X.T @ k, I


def sequential(A, B, C, Q, R, ud, ref, fixed, bval):
    N = ref.shape[0]
    P = Q.copy()
    p = -Q @ ref[N - 1]
    Ks, ks = [None] * N, [None] * N
    for i in range(N - 1, -1, -1):
        Ks[i], ks[i], P, p, _ = stage(P, p, A, B, C, Q, R, ud, ref[i], fixed[i], bval[i])
    x = np.zeros(3)
    us, xs = [], [x]
    for i in range(N):
        u = Ks[i] @ x + ks[i]
        x = A @ x + B @ u + C
        us.append(u)
        xs.append(x)
    return np.array(us), np.array(xs)


def segmented(A, B, C, Q, R, ud, ref, fixed, bval, S):
    N = ref.shape[0]
    bnd = [round(j * N / S) for j in range(S + 1)]
    seg = []
    for j in range(S):
        s, e = bnd[j], bnd[j + 1]
        last = j == S - 1
        P = Q.copy() if last else np.zeros((3, 3))
        p = -Q @ ref[N - 1] if last else np.zeros(3)
        Phi = np.eye(3)
        psi = np.zeros(3)
        Gam = np.zeros((3, 3))
        K, k, F = {}, {}, {}
        for i in range(e - 1, s - 1, -1):
            K[i], k[i], Pn, pn, I = stage(P, p, A, B, C, Q, R, ud, ref[i], fixed[i], bval[i])
            W = Phi @ B
            F[i] = -I @ W.T
            psi = Phi @ (B @ k[i] + C) + psi
            Gam = Gam + W @ F[i]
            Phi = Phi @ (A + B @ K[i])
            P, p = Pn, pn
        seg.append(dict(s=s, e=e, P=P, a=p, Phi=Phi, psi=psi, Gam=Gam, K=K, k=k, F=F))
    # Riccati over the segment ends: lam_{j-1} = M_j x_s^(j) + m_j
    M = seg[S - 1]["P"].copy()
    m = seg[S - 1]["a"].copy()
    T = [None] * S  # lam_j = T_j x_s^(j) + t_j  (j <= S-2)
    for j in range(S - 2, -1, -1):
        sj = seg[j]
        Ph, ps, Ga = sj["Phi"], sj["psi"], sj["Gam"]
        Z = np.linalg.inv(np.eye(3) - M @ Ga)
        Tj = Z @ M @ Ph
        tj = Z @ (M @ ps + m)
        T[j] = (Tj, tj)
        M = sj["P"] + Ph.T @ Tj
        m = sj["a"] + Ph.T @ tj
    xs_start = [np.zeros(3)]
    lam = []
    for j in range(S - 1):
        Tj, tj = T[j]
        lj = Tj @ xs_start[j] + tj
        lam.append(lj)
        sj = seg[j]
        xs_start.append(sj["Phi"] @ xs_start[j] + sj["psi"] + sj["Gam"] @ lj)
    lam.append(np.zeros(3))
    us = np.zeros((N, 2))
    xs = np.zeros((N + 1, 3))
    for j in range(S):
        sj = seg[j]
        x = xs_start[j]
        xs[sj["s"]] = x
        for i in range(sj["s"], sj["e"]):
            u = sj["K"][i] @ x + sj["k"][i] + sj["F"][i] @ lam[j]
            x = A @ x + B @ u + C
            us[i] = u
            xs[i + 1] = x
    return us, xs


def main():
    rng = np.random.default_rng(0)
    Q = np.diag([1.0, 1.0, 0.1])
    R = np.diag([0.1, 0.1])
    ud = np.array([4.5, 0.0])
    worst = 0.0
    for trial in range(300):
        N = int(rng.choice([4, 8, 20, 30, 40, 48]))
        S = int(rng.choice([2, 4, 8]))
        if S > N:
            continue
        A, B, C = model(rng, N, heading=bool(trial % 2))
        ref = np.cumsum(rng.normal(0, 0.05, (N, 3)), 0)
        ref[:, 0] += np.arange(1, N + 1) * 0.04
        fixed = rng.random((N, 2)) < rng.choice([0.0, 0.2, 0.6, 1.0])
        bval = np.stack([rng.choice([-1.0, 4.5], N), rng.choice([-0.43, 0.43], N)], 1)
        u1, x1 = sequential(A, B, C, Q, R, ud, ref, fixed, bval)
        u2, x2 = segmented(A, B, C, Q, R, ud, ref, fixed, bval, S)
        err = max(np.abs(u1 - u2).max() / max(1, np.abs(u1).max()), np.abs(x1 - x2).max() / max(1, np.abs(x1).max()))
        worst = max(worst, err)
    print(f"segmented vs sequential Riccati, 300 random problems: max rel err {worst:.2e}")
    assert worst < 1e-10


if __name__ == "__main__":
    main()
