"""tests/golden/stats_<name>.npz: the reference's get_average (Coop-MH-PPO-scalable.py:1550-1675)
on the deterministic-evaluation trajectories of tests/golden/eval_*.npz (the reference's own
Env_rollout.iterations output on the shipped weights).

The function (the first `def get_average` of the script, AST-extracted, unmodified) runs on
the fixture's `obs` reshaped as the script's cell does (:1081-1091), with:
  * `env` = a namespace with the fixture's nb_car / nb_ped / nb_lines;
  * `info_co2` = a no-op: its input LDV.csv is not shipped with the reference;
  * `torch` / `np` = thin recorders that pass every call through and record the result of
    each torch.mean / torch.std / np.mean / np.std call, in call order, and `print` =
    a recorder of its raw arguments — the statistics at full precision instead of the
    printed 2-decimal text.
Stored: the recorded values under the names of the quantities the reference prints.
"""
import ast
import builtins
import contextlib
import glob
import io
import os
import sys
import types

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import refclasses  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..")
# torch.mean / torch.std calls of get_average in call order (:1552-1668)
TORCH_CALLS = ["mean_speed_car0", "std_speed_car0", "mean_abs_acc_car0", "std_acc_car0", "mean_abs_speed_ped0",
               "std_abs_speed_ped0", "mean_speed_yielding_cars", "std_speed_yielding_cars",
               "mean_pass_time_yielding_cars", "mean_pass_time_cars", "mean_pass_time_peds", "interaction_cost",
               "interaction_cost_max", "std_pass_time_yielding_cars", "std_pass_time_cars", "std_pass_time_peds"]
NP_CALLS = ["mean_waiting_time", "std_waiting_time", "could_stop_share"]
PRINTS = {"Yield decision: ": "yield_share", "Go first decision: ": "go_share",
          "Scenario 1 1: ": "scenario_yield_yield", "Scenario -1 -1: ": "scenario_go_go",
          "Scenario -1 1: ": "scenario_go_yield", "Scenario 1 -1: ": "scenario_yield_go"}


def load_get_average():
    src = open(refclasses.SCRIPT).read().replace("\r", "")
    tree = ast.parse(src)
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "get_average")
    return compile(ast.Module(body=[fn], type_ignores=[]), "<reference get_average>", "exec")


def run(path):
    g = np.load(path)
    variant = str(g["variant"])
    nc, npd, nl = int(g["nb_car"]), int(g["nb_ped"]), int(g["nb_lines"])
    states = torch.tensor(g["obs"], dtype=torch.float)
    S = 2 * nl if variant == "scalable" else nc
    cw, ew = (7, 4) if variant == "scalable" else (6, 3)
    lim_car, lim_env, lim_ped = cw * S, ew, 9 * npd
    ep_car = states[:, :lim_car].reshape(-1, S, cw)                 # :1085-1086
    ep_env = states[:, lim_car:lim_car + lim_env].reshape(-1, lim_env)
    ep_ped = states[:, lim_car + lim_env:lim_car + lim_env + lim_ped].reshape((-1, npd, 9))
    ep_cross = ep_env[:, 0]
    rec_t, rec_n, rec_p = [], [], []

    def rec(store, fn):
        def f(*a, **k):
            r = fn(*a, **k)
            store.append(float(r))
            return r
        return f

    tproxy = types.SimpleNamespace(**{k: getattr(torch, k) for k in dir(torch) if not k.startswith("__")})
    tproxy.mean, tproxy.std = rec(rec_t, torch.mean), rec(rec_t, torch.std)
    nproxy = types.SimpleNamespace(**{k: getattr(np, k) for k in dir(np) if not k.startswith("__")})
    nproxy.mean, nproxy.std = rec(rec_n, np.mean), rec(rec_n, np.std)

    def pr(*a, **k):
        rec_p.append(a)

    ns = dict(torch=tproxy, np=nproxy, states=states, env=types.SimpleNamespace(nb_car=nc, nb_ped=npd, nb_lines=nl),
              info_co2=lambda *a, **k: None, LDV=None, math=__import__("math"), print=pr, sum=builtins.sum)
    exec(load_get_average(), ns)
    with contextlib.redirect_stdout(io.StringIO()):
        ns["get_average"](ep_car, ep_ped, ep_cross)
    assert len(rec_t) == len(TORCH_CALLS) and len(rec_n) == len(NP_CALLS), (len(rec_t), len(rec_n))
    out = dict(variant=variant, nb_car=nc, nb_ped=npd, nb_lines=nl, eval_fixture=os.path.basename(path))
    out.update({k: np.float64(v) for k, v in zip(TORCH_CALLS, rec_t)})
    out.update({k: np.float64(v) for k, v in zip(NP_CALLS, rec_n)})
    for a in rec_p:
        if a and isinstance(a[0], str) and a[0] in PRINTS:
            out[PRINTS[a[0]]] = np.float64(float(a[1]))
    return out


def main():
    for path in sorted(glob.glob(os.path.join(OUT, "eval_*.npz"))):
        g = np.load(path)
        if str(g["variant"]) != "scalable":  # get_average is the scalable script's cell
            continue
        name = os.path.basename(path)[5:-4]
        d = run(path)
        np.savez_compressed(os.path.join(OUT, f"stats_{name}.npz"), **d)
        print(name, {k: round(float(v), 5) for k, v in d.items() if k not in ("eval_fixture", "variant")})


if __name__ == "__main__":
    main()
