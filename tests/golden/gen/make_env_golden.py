"""Generate tests/golden/env_<name>.npz from the reference envs (build container only).

Per env e: its own CPython random stream seeded `random.seed(seed_base + e)`,
one reset, then T steps of forced actions.  Actions are float32 values promoted
to float64 exactly as the reference rollout passes them (Coop-MH-PPO-scalable.py
:454-460).  Light policies per env: constant per episode (what the reference
rollout does), random per step, and zeros, so every detection branch runs.
Run:  python3 tests/golden/gen/make_env_golden.py
"""
import contextlib
import io
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import refharness as R  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")

# name: (variant, nb_car, nb_ped, nb_lines, n_envs, seed_base, steps)
CASES = {
    "naif_111": ("naif", 1, 1, 1, 8, 100, 80),
    "coop_212": ("coop", 2, 1, 2, 8, 200, 80),
    "coop_422": ("coop", 4, 2, 2, 8, 250, 80),
    "4cars_412": ("4cars", 4, 1, 2, 8, 300, 80),
    "scalable_814": ("scalable", 8, 1, 4, 8, 400, 80),
    "scalable_432": ("scalable", 4, 3, 2, 8, 450, 80),
    "coop_133": ("coop", 1, 3, 3, 6, 500, 80),
    "naif_221": ("naif", 2, 2, 1, 6, 550, 80),
    "4cars2_412": ("4cars2", 4, 1, 2, 8, 600, 80),
    "4cars2_222": ("4cars2", 2, 2, 2, 6, 650, 80),
    "stop_212": ("stop", 2, 1, 2, 8, 700, 80),
    "stop_422": ("stop", 4, 2, 2, 8, 750, 80),
}


def n_slots(variant, nb_car, nb_lines):
    """Action slots: acc + light per slot (4cars2: AVs and PPO-driven followers)."""
    if variant == "scalable":
        return 2 * nb_lines
    return 2 * nb_car if variant == "4cars2" else nb_car


EVENTS = ("Accident! : ", "Possible accident! ", "Small mistake - priority ? ", "Pedestrian is not waiting ",
          "Mauvais signal vert ")  # detection's prints (scalable :186,200,222,227,236), MHPPO_EV_* order


def count_events(text):
    """Per-message counts of the reference env's detection prints in captured stdout."""
    lines = text.splitlines()
    return [sum(1 for ln in lines if ln.startswith(m)) for m in EVENTS]


def run_case(variant, nb_car, nb_ped, nb_lines, n_envs, seed_base, steps, capture_events=False):
    S = n_slots(variant, nb_car, nb_lines)
    arng = np.random.default_rng(seed_base)
    envs, streams = [], []
    for e in range(n_envs):
        envs.append(R.make(variant, nb_car, nb_ped, nb_lines))
        streams.append(R.Stream(seed_base + e))
    obs0, mti0, obs, rew, rl, done, mti, dumps, acts = [], [], [], [], [], [], [], [], []
    for e in range(n_envs):
        with streams[e].active():
            s, _ = envs[e].reset()
        obs0.append(R.flat(s))
        mti0.append(streams[e].mti)
    modes = [e % 3 for e in range(n_envs)]  # 0 constant lights, 1 random lights, 2 mixed incl. zeros
    const_light = arng.choice([-1.0, 1.0], size=(n_envs, S))
    events = []
    for t in range(steps):
        o_t, r_t, l_t, d_t, m_t, x_t, a_t, ev_t = [], [], [], [], [], [], [], []
        for e in range(n_envs):
            acc = arng.uniform(-4.5, 2.5, size=S).astype(np.float32).astype(np.float64)
            if modes[e] == 0:
                light = const_light[e]
            elif modes[e] == 1:
                light = arng.choice([-1.0, 1.0], size=S)
            else:
                light = arng.choice([-1.0, 0.0, 1.0], size=S)
            a = np.concatenate([acc, light]).astype(np.float64)
            buf = io.StringIO()
            with streams[e].active(), contextlib.redirect_stdout(buf):
                s, r, d, _, _ = envs[e].step(a)
            ev_t.append(count_events(buf.getvalue()))
            o_t.append(R.flat(s))
            r_t.append(np.asarray(r, dtype=np.float64))
            l_t.append(np.asarray(envs[e].reward_light, dtype=np.float64))
            d_t.append(bool(d))
            m_t.append(streams[e].mti)
            x_t.append(R.dump(envs[e]))
            a_t.append(a)
        obs.append(o_t); rew.append(r_t); rl.append(l_t); done.append(d_t); mti.append(m_t)
        dumps.append(x_t); acts.append(a_t); events.append(ev_t)
    final_mt = np.array([np.array(st.state[1][:624], dtype=np.uint32) for st in streams])
    sw = lambda x: np.swapaxes(np.array(x), 0, 1)  # [T,E,...] -> [E,T,...]
    extra = dict(events=sw(events).astype(np.int16)) if capture_events else {}
    return dict(
        **extra, variant=variant, nb_car=nb_car, nb_ped=nb_ped, nb_lines=nb_lines, seed_base=seed_base,
        obs0=np.array(obs0), mti0=np.array(mti0), actions=sw(acts), obs=sw(obs), rewards=sw(rew),
        reward_light=sw(rl), done=sw(done), mti=sw(mti), dump=sw(dumps), final_mt=final_mt,
        final_mti=np.array([st.mti for st in streams]),
    )


def main():
    for name, case in CASES.items():
        d = run_case(*case)
        path = os.path.join(OUT, f"env_{name}.npz")
        np.savez_compressed(path, **d)
        print(name, {k: getattr(v, "shape", v) for k, v in d.items() if k in ("obs", "dump")},
              os.path.getsize(path))


if __name__ == "__main__":
    main()
