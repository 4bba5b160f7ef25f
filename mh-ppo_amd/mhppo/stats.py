"""Evaluation statistics of the paper cells (`get_average`, Coop-MH-PPO-scalable.py:1550-1675),
over the deterministic-evaluation trajectories Algo_PPO.evaluate returns.

Input: `states`, the float32 [rows, obs_dim] observations evaluate() returns (gym-sorted
car | env | ped, one row per step), reshaped as the notebook cell does (:1081-1091):
ep_car [rows, S, car_width], ep_ped [rows, P, 9], ep_cross = env[:, 0].  Episodes are the
maximal runs of rows with an equal ep_cross, scanned pairwise (t, t+1) exactly as the
reference's while-loops do (:1593-1640):
  pedestrian p  waiting_time  += 0.3 per pair with |Sy| == cross at t and t+1, and again per
                              pair with |Sy| == 0 at t and t+1 (:1598-1603)
                ped_leave     = 0.3 k of the LAST pair k where Sy*dir crosses cross (:1604-1606),
                              the episode's span when there is none (or it is 0) (:1608-1609)
  car i < nb_car  no-interaction time (25 - Sc)/Vc at the first row (:1619)
                could_stop    when the light at row 1 is go (< 0) (:1620-1624)
                car_leave     = 0.3 k of the LAST pair where Sc - max_p Sx - 25 crosses 0 (:1630-1631)
                speed_cars / temp_cars for cars that yield (light == 1 at row 1) (:1627-1634)
                decision      = the light at the last pair's first row (:1626, :1640)
Statistics as the cell prints them (:1641-1673): float32 torch means / unbiased stds,
numpy population statistics for the waiting times, decision shares per EPISODE (the
reference divides the count of car decisions by the number of episodes).  The CO2
leg (info_co2, :1524-1548) needs LDV.csv, which the reference does not ship: not built.

The arithmetic is vectorised torch on the states' device (float32 comparisons and
differences, as the reference's float32 tensor elements compute them; the 0.3-step
sums in float64, as its Python floats do).
"""
import numpy as np
import torch

_CAR_W = {"scalable": 7, "coop": 6, "naif": 6, "stop": 6}
_ENV_W = {"scalable": 4, "coop": 3, "naif": 3, "stop": 3}


def _repeated_add(step, n):
    """w[k] = step + step + ... (k Python float additions, left to right)."""
    w = np.zeros(n + 1)
    acc = 0.0
    for k in range(1, n + 1):
        acc += step
        w[k] = acc
    return w


def split_states(states, variant, nb_car, nb_ped, nb_lines):
    """ep_car, ep_env, ep_ped, ep_cross as the reference cell builds them (:1081-1091)."""
    if variant not in _CAR_W:
        raise ValueError(f"get_average is defined for the scalable/coop/naif/stop drivers' observation "
                         f"layout (car|env|ped), not {variant!r}")
    S = 2 * nb_lines if variant == "scalable" else nb_car
    cw, ew = _CAR_W[variant], _ENV_W[variant]
    st = torch.as_tensor(states, dtype=torch.float32)
    lim_car, lim_ped = cw * S, 9 * nb_ped
    ep_car = st[:, :lim_car].reshape(-1, S, cw)
    ep_env = st[:, lim_car:lim_car + ew]
    ep_ped = st[:, lim_car + ew:lim_car + ew + lim_ped].reshape(-1, nb_ped, 9)
    return ep_car, ep_env, ep_ped, ep_env[:, 0]


def get_average(states, variant, nb_car, nb_ped, nb_lines, dt_step=0.3):
    """The statistics get_average prints, as a dict of Python floats (CO2 excluded)."""
    ep_car, _, ep_ped, cross = split_states(states, variant, nb_car, nb_ped, nb_lines)
    dev = ep_car.device
    R = cross.shape[0]
    if R < 2:
        raise ValueError("need at least two rows")
    out = {
        "mean_speed_car0": torch.mean(ep_car[:, 0, 1]).item(), "std_speed_car0": torch.std(ep_car[:, 0, 1]).item(),
        "mean_abs_acc_car0": torch.mean(torch.abs(ep_car[:, 0, 0])).item(),
        "std_acc_car0": torch.std(ep_car[:, 0, 0]).item(),
        "mean_abs_speed_ped0": torch.mean(torch.abs(ep_ped[:, 0, 1])).item(),
        "std_abs_speed_ped0": torch.std(torch.abs(ep_ped[:, 0, 1])).item(),
    }
    # ---- episodes: maximal runs of equal cross; pair t = (t, t+1) belongs to the run of t
    same = cross[:-1] == cross[1:]                       # [R-1]
    starts = [0]
    brk = torch.nonzero(~same).reshape(-1).cpu().tolist()  # pair t breaks the run: next run starts at t+1
    starts += [b + 1 for b in brk]
    ends = [s - 1 for s in starts[1:]] + [R - 1]         # last row of each run
    seg = [(a, b) for a, b in zip(starts, ends) if a < R - 1]   # the loop runs while t_init + 1 < R
    if any(b == a for a, b in seg):
        raise ValueError("an episode of a single row (equal cross values across episodes?)")
    E = len(seg)
    a_idx = torch.tensor([a for a, _ in seg], device=dev)
    b_idx = torch.tensor([b for _, b in seg], device=dev)
    span = (b_idx - a_idx)                               # pairs per episode
    # pair -> episode id, k = t - t_init, for pairs inside an episode
    pair_ep = torch.full((R - 1,), -1, dtype=torch.long, device=dev)
    first = torch.cumsum(span, 0) - span                 # each episode's first pair in the packed list
    local = torch.arange(int(span.sum()), device=dev) - torch.repeat_interleave(first, span)
    pair_ep[torch.repeat_interleave(a_idx, span) + local] = torch.repeat_interleave(torch.arange(E, device=dev), span)
    inside = pair_ep >= 0
    t = torch.arange(R - 1, device=dev)
    k = t - a_idx[pair_ep.clamp(min=0)]
    W = torch.tensor(_repeated_add(dt_step, R), dtype=torch.float64, device=dev)
    kdt = torch.tensor([i * dt_step for i in range(R)], dtype=torch.float64, device=dev)  # (t - t_init) * 0.3

    def last_k(cond):  # [E] last k with cond (0 when none), as python's overwriting assignment
        kk = torch.where(cond & inside, k, torch.zeros_like(k))
        return torch.zeros(E, dtype=torch.long, device=dev).scatter_reduce(0, pair_ep.clamp(min=0), kk, "amax")

    def count(cond):
        return torch.zeros(E, dtype=torch.long, device=dev).index_add_(0, pair_ep.clamp(min=0),
                                                                        (cond & inside).long())

    ped_leave, waiting, fcn_ped, direction = [], [], [], []
    for p in range(nb_ped):
        sy, dr = ep_ped[:, p, 3], ep_ped[:, p, 8]
        c1 = (torch.abs(sy[:-1]) == cross[:-1]) & (torch.abs(sy[1:]) == cross[1:])
        c2 = (torch.abs(sy[:-1]) == 0) & (torch.abs(sy[1:]) == 0)
        wt = W[count(c1) + count(c2)]
        c3 = ((sy[:-1] * dr[:-1]) < cross[:-1]) & ((sy[1:] * dr[1:]) >= cross[1:])
        lk = last_k(c3)
        pl = torch.where(lk == 0, kdt[span], kdt[lk])
        ped_leave.append(pl)
        waiting.append(wt)
        fcn_ped.append(pl - wt)
        direction.append((-dr[a_idx] / 2.0 + 0.5).long())
    maxsx = torch.max(ep_ped[:, :, 2], dim=1).values     # max over pedestrians of Sx, per row
    car_leave, fcn_car, decision, light1 = [], [], [], []
    could_stop, speed_cars, temp_cars = [], [], []
    for i in range(nb_car):
        sc, vc, li = ep_car[:, i, 3], ep_car[:, i, 1], ep_car[:, i, 4]
        fcn_car.append((25.0 - sc[a_idx]) / vc[a_idx])
        l1 = li[a_idx + 1]
        light1.append(l1)
        cs = ((-sc[a_idx] - (vc[a_idx] * vc[a_idx] / 8.0 + vc[a_idx])) > 0.0).long()
        could_stop.append(torch.where(l1 < 0.0, cs, torch.full_like(cs, -1)))   # -1: not appended
        d0 = (sc[:-1] - maxsx[1:]) - 25
        d1 = (sc[1:] - maxsx[1:]) - 25
        c4 = (d0 < 0.0) & (d1 >= 0.0)
        lk = last_k(c4)
        car_leave.append(torch.where(lk == 0, kdt[span], kdt[lk]))
        decision.append(li[b_idx - 1])
        yields = (l1 == 1)[pair_ep.clamp(min=0)] & inside  # pair of an episode whose car i yields
        speed_cars.append((vc[:-1], yields))
        temp_cars.append((kdt[k.clamp(min=0)], yields & c4))
    # ---- lists in the reference's append order (episode-major; peds then cars)
    temp_peds = torch.stack(ped_leave, 1).reshape(-1)                      # [E*P]
    waits = torch.stack(waiting, 1).reshape(-1).cpu().numpy()
    fci = torch.cat([torch.stack(ped_leave, 1).float(), torch.stack(car_leave, 1).float()], 1)   # [E, P+nb_car]
    fcn = torch.cat([torch.stack(fcn_ped, 1).float(), torch.stack(fcn_car, 1).float()], 1)
    all_dec = torch.stack(decision, 1)                                      # [E, nb_car]
    all_tc = torch.stack(car_leave, 1).reshape(-1).float()

    def ordered(pairs):  # episode-major, car-major, pair order — the reference's list order
        vals = torch.stack([v for v, _ in pairs], 0)       # [nb_car, R-1]
        msk = torch.stack([m for _, m in pairs], 0)
        key = pair_ep.clamp(min=0).unsqueeze(0) * (nb_car * R) + torch.arange(nb_car, device=dev).unsqueeze(1) * R + t
        key = torch.where(msk, key, torch.full_like(key, -1)).reshape(-1)
        sel = torch.nonzero(key >= 0).reshape(-1)
        order = torch.argsort(key[sel])
        return vals.reshape(-1)[sel][order]

    sp = ordered(speed_cars).float()
    tc = ordered(temp_cars).float()
    cst = torch.stack(could_stop, 1).reshape(-1)
    cst = cst[cst >= 0].cpu().numpy()
    ic = torch.max(fci, dim=1, keepdim=True).values - torch.max(fcn, dim=1, keepdim=True).values
    n_ep = all_dec.shape[0]
    out.update({
        "mean_speed_yielding_cars": torch.mean(sp).item(), "std_speed_yielding_cars": torch.std(sp).item(),
        "interaction_cost": torch.mean(ic).item(), "interaction_cost_max": torch.mean(fci - fcn).item(),
        "mean_pass_time_yielding_cars": torch.mean(tc).item(), "std_pass_time_yielding_cars": torch.std(tc).item(),
        "mean_pass_time_cars": torch.mean(all_tc).item(), "std_pass_time_cars": torch.std(all_tc).item(),
        "mean_pass_time_peds": torch.mean(temp_peds.float()).item(),
        "std_pass_time_peds": torch.std(temp_peds.float()).item(),
        "yield_share": int((all_dec == 1).sum()) / n_ep, "go_share": int((all_dec == -1).sum()) / n_ep,
        "mean_waiting_time": float(np.mean(waits)), "std_waiting_time": float(np.std(waits)),
        "could_stop_share": float(np.mean(cst)) if cst.size else float("nan"),
        "episodes": n_ep,
    })
    if nb_car == 2:
        s = all_dec.sum(1)
        out.update({"scenario_yield_yield": int((s == 2).sum()) / n_ep, "scenario_go_go": int((s == -2).sum()) / n_ep,
                    "scenario_go_yield": int(((all_dec[:, 0] == -1) & (all_dec[:, 1] == 1)).sum()) / n_ep,
                    "scenario_yield_go": int(((all_dec[:, 0] == 1) & (all_dec[:, 1] == -1)).sum()) / n_ep})
    return out
