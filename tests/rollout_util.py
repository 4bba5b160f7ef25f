"""Shared helpers for the rollout parity tests: bucket per-(env, slot) rollout
outputs the way Env_rollout.iterations_rand appends them (:489-507)."""
import numpy as np


def bucket(out, scalable):
    """out: dict of per-env arrays (oracle.rollout or GPU buffers as numpy)."""
    N, S, P = out["a_d"].shape
    res = {k: [] for k in ("obs_cross", "act_cross", "logp_cross", "rew_cross", "obs_wait", "act_wait", "logp_wait",
                           "rew_wait", "obs_choice", "act_choice", "logp_choice", "rew_choice")}
    for e in range(N):
        action_d = 2 * out["a_d"][e].reshape(-1).astype(np.int64) - 1
        for i in range(S):
            if scalable and not out["exist"][e, i]:
                continue
            b = "cross" if action_d[i] <= 0 else "wait"
            res["obs_" + b].append(out["obs_c"][e, i])
            res["act_" + b].append(out["act"][e, i])
            res["logp_" + b].append(out["logp"][e, i])
            res["rew_" + b].append(out["rew"][e, i])
            c = out["closest"][e, i]
            res["obs_choice"].append(out["feat_d"][e, i, c][None])
            res["act_choice"].append(np.array([out["a_d"][e, i, c]], np.float64))
            res["logp_choice"].append(np.array([out["logp_d"][e, i, c]], np.float64))
            res["rew_choice"].append(np.array([out["ep_min"][e, i]]))
    return {k: (np.concatenate(v) if v else np.zeros((0,))) for k, v in res.items()}


def returns(rew_flat, T=80, gamma=0.99):
    r = rew_flat.reshape(-1, T)
    out = np.zeros_like(r, dtype=np.float32)
    g = np.zeros(r.shape[0])
    for t in range(T - 1, -1, -1):
        g = r[:, t] + gamma * g
        out[:, t] = g.astype(np.float32)
    return out.reshape(-1)
