"""Env_rollout / Algo_PPO with the reference's API, running on the MI355X path.

Drop-in surface of Coop-MH-PPO-scalable.py §3-§4 (:96-1001) and the coop
driver (Coop-MH-PPO.ipynb cell 0): same class names, constructor arguments,
method names, hyper-parameter defaults and checkpoint file names/keys.  The
environment is a VecCrosswalk of N envs: one `train` iteration plays one
80-step episode in every env (the reference plays 26 episodes of one env for
batch_size=2048), then runs the same 10 + 10 full-batch epochs.
"""
import contextlib
import os

import numpy as np
import torch
import torch.distributed as dist

from . import _lib, ppo
from .env import VecCrosswalk
from .models import Model_PPO
from .rollout import RolloutGPU, bucket_segments

PREFIX = {"scalable": "pappo-scalable-coop", "coop": "pappo-coop", "4cars": "pappo-coop-4cars", "naif": "pappo-acc6"}


def _rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def _rank_path(path):
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return f"{path}.rank{dist.get_rank()}"
    return path


def _venv(env):
    return env.venv if hasattr(env, "venv") else env


class Env_rollout:
    """Batched Env_rollout (:96-684): collects one episode per env per call."""

    def __init__(self, env, nb_cars, max_steps, dt):
        self.env = _venv(env)
        self.nb_cars = nb_cars
        self.dt = dt
        self.max_steps = max_steps
        self.shape_env = 2 + 9 + 2
        self.gpu = RolloutGPU(self.env, T=max_steps)
        self.shape_env_d = self.gpu.dc
        self.seed = 0
        self.iteration = 0
        self.fix_bucket = False  # opt-in bug fix (Algo_PPO.fix_bucket)
        self.env.reset(want_obs=False)  # the reference's __init__ resets the env (:107)
        self.batch = None
        self.cross = self.wait = self.choice = None

    def reset(self):
        """(:125-144) clears the batches and resets the env, consuming that reset's draws
        in every env's random stream exactly as the reference does."""
        self.env.reset(want_obs=False)
        self.batch = None
        self.cross = self.wait = self.choice = None

    def iterations(self, actor_net_cross, actor_net_wait, actor_net_choice, nbr_episodes, choix=False):
        """Deterministic evaluation (:152-252) of `nbr_episodes` consecutive episodes in every
        env; returns (obs, acts, rews_c, rews_d, waiting_time) env-major (see RolloutGPU.evaluate).
        choix=True: the scripted choix_test scenario (:629-633) after every reset."""
        with torch.no_grad():
            return self.gpu.evaluate(actor_net_cross, actor_net_wait, actor_net_choice, nbr_episodes, choix=choix)

    def iterations_rand(self, actor_net_cross, actor_net_wait, actor_net_choice, cov_mat=None, cov_mat_d=None,
                        batch_size=None, random_rate=0.0, forced_choice=None, eps_tape=None):
        """One episode in every env (:357-517); buckets the segments like :489-507."""
        with torch.no_grad():
            self.batch = self.gpu.collect(actor_net_cross, actor_net_wait, actor_net_choice, seed=self.seed,
                                          iteration=self.iteration, forced_choice=forced_choice, eps_tape=eps_tape)
        self.iteration += 1
        # NaN policy outputs raise, as torch.distributions does in the reference: the status word
        # comes back with the bucket sizes (the iteration's one host sync before the update)
        self.cross, self.wait, self.choice = bucket_segments(self.batch, fix_bucket=self.fix_bucket,
                                                             status=self.gpu.status)
        return self.batch

    # reference-named views of the collected batch
    @property
    def batch_obs_cross(self):
        return self.cross["obs"]

    @property
    def batch_obs_wait(self):
        return self.wait["obs"]

    @property
    def batch_obs_choice(self):
        return self.choice["obs"]

    def futur_rewards(self):
        """(:658-684) reward-to-go per bucket (float32); choice = episodic min."""
        return self.cross["ret"], self.wait["ret"], self.choice["ret"]

    def immediate_rewards(self):
        """(:635-656)"""
        return self.cross["rew"].float(), self.wait["rew"].float(), self.choice["ret"]


class Algo_PPO:
    """Multi-head PPO (:698-1001)."""

    def __init__(self, policy_class, env, **hyperparameters):
        self._init_hyperparameters(hyperparameters)
        venv = _venv(env)
        self.venv = venv
        self.max_steps = venv.max_episode
        S = venv.n_slots
        if not hasattr(self, "num_states_c"):
            self.num_states_c = 13
        if not hasattr(self, "num_states_d"):
            self.num_states_d = _lib.lib().mhppo_choice_dim(venv.handle)
        if not hasattr(self, "num_actions"):
            self.num_actions = 1
        if not hasattr(self, "mean"):
            self.mean = (venv.cfg.car_b[2] + venv.cfg.car_b[0]) / 2.0   # :1044
        if not hasattr(self, "std"):
            self.std = (venv.cfg.car_b[2] - venv.cfg.car_b[0]) / 2.0    # :1045
        if not hasattr(self, "dt"):
            self.dt = venv.dt
        dev = venv.device
        self.actor_net_cross = policy_class(self.num_states_c, self.num_actions, 1, nb_car=S, mean=self.mean,
                                            std=self.std).to(dev)
        self.actor_net_wait = policy_class(self.num_states_c, self.num_actions, 1, nb_car=S, mean=self.mean,
                                           std=self.std).to(dev)
        self.actor_net_choice = policy_class(self.num_states_d, 2, 2).to(dev)
        self.critic_net_cross = policy_class(self.num_states_c, 1, 0).to(dev)
        self.critic_net_wait = policy_class(self.num_states_c, 1, 0).to(dev)
        self.critic_net_choice = policy_class(self.num_states_d, 1, 0).to(dev)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            for net in self.nets():  # replicas start identical (rank 0's init)
                for p in net.parameters():
                    dist.broadcast(p.data, src=0)
        # every net's flat gradient in one contiguous buffer: one in-place all-reduce per
        # joint epoch under data parallelism (mhppo.ppo.GradBucket)
        # (actors first, then critics: the first and last steps of the epoch pipeline, which train
        # only the critics / only the actors, reduce one contiguous span too)
        self.grad_bucket = ppo.GradBucket([self.actor_net_cross, self.actor_net_wait, self.actor_net_choice,
                                           self.critic_net_cross, self.critic_net_wait, self.critic_net_choice],
                                          dev)
        # one fused Adam launch per net and step on the GPU (the reference's default Adam
        # semantics: lr, betas (0.9, 0.999), eps 1e-8, no weight decay)
        A = (lambda params, lr: torch.optim.Adam(params, lr, fused=True)) if dev.type == "cuda" else torch.optim.Adam
        self.optimizer_critic_cross = A(self.critic_net_cross.parameters(), self.critic_lr)
        self.optimizer_critic_wait = A(self.critic_net_wait.parameters(), self.critic_lr)
        self.optimizer_critic_choice = A(self.critic_net_choice.parameters(), self.critic_d_lr)
        self.optimizer_actor_cross = A(self.actor_net_cross.parameters(), self.actor_lr)
        self.optimizer_actor_wait = A(self.actor_net_wait.parameters(), self.actor_lr)
        self.optimizer_actor_choice = A(self.actor_net_choice.parameters(), self.actor_d_lr)
        self.value_std = 0.5
        self.value_std_d = 0.1
        self.cov_var = torch.full(size=(self.num_actions,), fill_value=self.value_std)
        self.cov_mat = torch.diag(self.cov_var)
        self.cov_var_d = torch.full(size=(2 * S,), fill_value=self.value_std_d)
        self.cov_mat_d = torch.diag(self.cov_var_d)
        self.rollout = Env_rollout(venv, S, self.max_steps, self.dt)
        self.rollout.seed = getattr(self, "seed", 0)
        # reward curves (:886-892).  While train() runs with verbose=False they lag by one
        # iteration: an iteration's sums are read back asynchronously and appended at the next
        # iteration (or at the end of train()); curves() / save_checkpoint() flush them first.
        self.ep_reward_cross, self.ep_reward_wait, self.ep_reward_choice = [], [], []
        self.ep_scenario_balance = []
        self._pending_curves = []  # (pinned sums, event, m_c, m_w, m_d) not yet appended
        self.last_losses = {}

    def nets(self):
        return [self.actor_net_cross, self.actor_net_wait, self.actor_net_choice, self.critic_net_cross,
                self.critic_net_wait, self.critic_net_choice]

    def _init_hyperparameters(self, hyperparameters):
        """(:919-933) defaults; overrides set as attributes (the reference uses exec)."""
        self.num_algo = 1
        self.total_loop = 0
        self.batch_size = 2048
        self.gamma = 0.99
        self.critic_lr = 1e-3
        self.actor_lr = 3e-4
        self.critic_d_lr = 1e-3
        self.actor_d_lr = 3e-4
        self.verbose = True
        # opt-in bug fixes, off for parity: bucket cars by their closest
        # pedestrian's decision; per-row choice loss (not the M x M broadcast).  The scalable
        # lane fix is an env option: VecCrosswalk(..., fix_scalable_lanes=True).
        self.fix_bucket = False
        self.fix_choice_loss = False
        # all heads trained on the exact f32-MFMA kernel (k-ordered fmaf sums) instead of the
        # default bf16x3 split-precision one (f32-level products at 2.67x the f32-MFMA ceiling)
        self.exact_f32 = False
        # reward curves written to load_model/parameters at the end of train() (:908-916)
        self.save_curves = True
        for k, v in hyperparameters.items():
            setattr(self, k, v)

    def update(self):
        """10 epochs of cross+wait, then 10 epochs of choice (:868-882) on the collected batch,
        run as 10 joint epochs of the three independent heads (mhppo.ppo.train_epoch: same
        results, two collectives per epoch under data parallelism).  The global row counts
        and choice action counts take one all-reduce and one host sync per iteration."""
        r = self.rollout
        dev = self.venv.device
        c, w, d = r.cross, r.wait, r.choice
        with (torch.cuda.device(dev) if dev.type == "cuda" else contextlib.nullcontext()):
            counts = d.get("counts")  # queued with the bucketing, before its host sync
            if counts is None:
                counts = torch.stack([(d["act"] == 0).sum(), (d["act"] == 1).sum()]).to(torch.float64)
            if ppo._dp():  # global row counts: one all-reduce and one host sync
                loc = torch.cat([torch.tensor([c["ret"].numel(), w["ret"].numel(), d["ret"].numel()],
                                              dtype=torch.float64, device=dev), counts])
                ppo._allreduce_(loc)
                m_c, m_w, m_d = loc[:3].tolist()
                counts = loc[3:5]
            else:  # the local counts are the global ones, known on the host: no sync
                m_c, m_w, m_d = float(c["ret"].numel()), float(w["ret"].numel()), float(d["ret"].numel())
            heads, names = [], []
            if m_c > 0:  # the reference trains a continuous head only on a non-empty batch (:869, :874)
                heads.append(ppo.Head("c", self.actor_net_cross, self.critic_net_cross, self.optimizer_actor_cross,
                                      self.optimizer_critic_cross, c["obs"], c["act"], c["logp"], c["ret"], m_c,
                                      exact=self.exact_f32))
                names.append("cross")
            if m_w > 0:
                heads.append(ppo.Head("c", self.actor_net_wait, self.critic_net_wait, self.optimizer_actor_wait,
                                      self.optimizer_critic_wait, w["obs"], w["act"], w["logp"], w["ret"], m_w,
                                      exact=self.exact_f32))
                names.append("wait")
            if m_d > 0:  # never empty in the reference (>= 1 existing car per episode); it would raise there
                heads.append(ppo.Head("d", self.actor_net_choice, self.critic_net_choice, self.optimizer_actor_choice,
                                      self.optimizer_critic_choice, d["obs"], d["act"], d["logp"], d["ret"], m_d,
                                      counts, per_row=self.fix_choice_loss, exact=self.exact_f32))
                names.append("choice")
            losses = ppo.train_epochs(heads, 10, self.grad_bucket) if heads else None
        if self.verbose and losses is not None:
            div = {"cross": (m_c, m_c), "wait": (m_w, m_w), "choice": (m_d * m_d, m_d)}
            if self.fix_choice_loss:
                div["choice"] = (m_d, m_d)
            self.last_losses = {k: (float(a.item()) / div[k][0], float(b.item()) / div[k][1])
                                for k, (a, b) in zip(names, losses)}
        return m_c, m_w, m_d

    def evaluate(self, nbr_episodes, choix=False):
        """(:738-747) rollout.reset() then the deterministic iterations; with N envs every env
        plays `nbr_episodes` episodes (N * nbr_episodes in total, env-major)."""
        self.rollout.reset()
        return self.rollout.iterations(self.actor_net_cross, self.actor_net_wait, self.actor_net_choice,
                                       nbr_episodes, choix=choix)

    def get_average(self, states):
        """The paper cell's evaluation statistics (get_average, :1550-1675; CO2 leg excluded)
        over `states`, the observations evaluate() returned (mhppo.stats)."""
        from .stats import get_average
        v = self.venv
        return get_average(states, v.variant, v.nb_car, v.nb_ped, v.nb_lines)

    def train(self, nb_loop, replay=None):
        """(:854-917): per iteration rollout.reset() -> one episode per env -> 10 + 10 epochs
        -> reward curves -> rollout.reset() (both resets consume env draws, as in the
        reference); at the end the curves go to load_model/parameters/*.npy (:908-916).
        replay (parity tests): one (forced_choice, eps_tape) pair per iteration, the
        recorded Categorical and MVN draws replayed instead of Philox noise."""
        self.rollout.fix_bucket = self.fix_bucket
        for ep in range(nb_loop):
            self.rollout.reset()
            fc, et = replay[ep] if replay is not None else (None, None)
            self.rollout.iterations_rand(self.actor_net_cross, self.actor_net_wait, self.actor_net_choice,
                                         self.cov_mat, self.cov_mat_d, self.batch_size, forced_choice=fc,
                                         eps_tape=et)
            m_c, m_w, m_d = self.update()
            rc, rw, rd = self.rollout.immediate_rewards()
            dev = self.venv.device
            sums = torch.stack([rc.double().sum(), rw.double().sum(), rd.double().sum()]).to(dev)
            ppo._allreduce_(sums)
            if dev.type == "cuda":
                # the reward curves take the sums without a host sync here: an asynchronous copy to
                # pinned memory, appended once it has landed (next iteration, or the end of train)
                host = torch.empty(3, dtype=torch.float64, pin_memory=True)
                host.copy_(sums, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(dev))
                self._pending_curves.append((host, ev, m_c, m_w, m_d))
            else:  # (CPU test doubles of the rollout: tests/test_dp_gloo.py)
                self._pending_curves.append((sums.clone(), None, m_c, m_w, m_d))
            if self.verbose:
                self._flush_curves()
            if self.verbose and _rank() == 0:
                print("Episode * {} * And Number of steps is ==> {}".format(ep, ep * self.batch_size))
                print("Average Cross reward is ==> {}, Average Wait reward is ==> {}".format(
                    np.mean(self.ep_reward_cross[-10:]) if self.ep_reward_cross else float("nan"),
                    np.mean(self.ep_reward_wait[-10:]) if self.ep_reward_wait else float("nan")))
                print("Average Choice reward is ==> {}".format(np.mean(self.ep_reward_choice[-10:])))
                print("Number Cross is ==> {} and Number Wait is ==> {} ".format(int(m_c), int(m_w)))
            self.rollout.reset()
            self.total_loop = self.total_loop + 1
            if len(self._pending_curves) > 1:  # the previous iteration's sums landed long ago
                self._flush_curves(keep_last=True)
        self._flush_curves()
        if _rank() == 0 and self.save_curves:
            self.save_reward_curves()
        if self.verbose and _rank() == 0:
            print("Complete")

    def _flush_curves(self, keep_last=False):
        """Append the reward-curve entries (rew_batch.mean() over the global batch, :886-892) of
        the iterations whose reward sums have been read back."""
        n = len(self._pending_curves) - (1 if keep_last else 0)
        for host, ev, m_c, m_w, m_d in self._pending_curves[:n]:
            if ev is not None:
                ev.synchronize()
            s = host.tolist()
            if m_c > 0:
                self.ep_reward_cross.append(s[0] / m_c)
            if m_w > 0:
                self.ep_reward_wait.append(s[1] / m_w)
            self.ep_reward_choice.append(s[2] / m_d if m_d > 0 else float("nan"))  # mean() of empty: NaN
            self.ep_scenario_balance.append([int(m_c), int(m_w)])
        del self._pending_curves[:n]

    def curves(self):
        """The reward curves with every pending entry appended: (cross, wait, choice, balance)."""
        self._flush_curves()
        return self.ep_reward_cross, self.ep_reward_wait, self.ep_reward_choice, self.ep_scenario_balance

    def _curve_path(self, name):
        pre = PREFIX.get(self.venv.variant, "pappo")
        return "load_model/parameters/{}-{:02d}-{}-step-{:03d}000.npy".format(pre, self.num_algo, name,
                                                                             int(self.total_loop / 1000))

    def save_reward_curves(self):
        """(:908-916) reward_cross / reward_wait / reward_choice / scenario_balance."""
        self._flush_curves()
        os.makedirs("load_model/parameters", exist_ok=True)
        for name, v in (("reward_cross", np.array(self.ep_reward_cross)), ("reward_wait", np.array(self.ep_reward_wait)),
                        ("reward_choice", np.array(self.ep_reward_choice)),
                        ("scenario_balance", np.array(self.ep_scenario_balance).reshape((-1, 2)))):
            with open(self._curve_path(name), "wb") as f:
                np.save(f, v)

    # --------------------------------------------------------------- checkpoints
    def _path(self, head, kind, num_algo, total_loop):
        pre = PREFIX.get(self.venv.variant, "pappo")
        return "load_model/weights/{}-{}-{:02d}-{}-step-{:03d}0.pth".format(pre, head, num_algo, kind,
                                                                           int(total_loop / 10))

    def loading(self, num_algo, total_loop):
        """(:935-955) torch state_dicts, loaded without executing anything from the file."""
        self.num_algo, self.total_loop = num_algo, total_loop
        for head in ("cross", "wait", "choice"):
            for kind in ("actor", "critic"):
                net = getattr(self, f"{kind}_net_{head}")
                sd = torch.load(self._path(head, kind, num_algo, total_loop), map_location=self.venv.device,
                                weights_only=True)
                net.load_state_dict(sd)

    def loading_curriculum(self, num_actor, num_algo, total_loop):
        """(:957-983) load one head's actor + critic: 0 cross, 1 wait, 2 choice."""
        self.total_loop = total_loop
        head = ("cross", "wait", "choice")[num_actor]
        for kind in ("actor", "critic"):
            net = getattr(self, f"{kind}_net_{head}")
            net.load_state_dict(torch.load(self._path(head, kind, num_algo, total_loop),
                                           map_location=self.venv.device, weights_only=True))

    # Checkpoint/resume beyond the reference: the reference keeps only
    # weights; an exact resume also needs the Adam moments, every env's state and random
    # stream, the rollout noise counter and the reward curves.
    def _optimizers(self):
        return {f"{k}_{h}": getattr(self, f"optimizer_{k}_{h}") for h in ("cross", "wait", "choice")
                for k in ("actor", "critic")}

    def save_checkpoint(self, path):
        """Everything needed to continue training bit-identically.  Under data parallelism
        every rank writes `path.rank<r>` (its env shard differs; nets/Adam are replicated)."""
        self._flush_curves()  # the newest iteration's curve entries may still be in flight
        ck = {
            "nets": {f"{k}_{h}": getattr(self, f"{k}_net_{h}").state_dict() for h in ("cross", "wait", "choice")
                     for k in ("actor", "critic")},
            "optim": {k: o.state_dict() for k, o in self._optimizers().items()},
            "env": self.venv.state_dict(),
            "rollout": {"iteration": int(self.rollout.iteration), "seed": int(self.rollout.seed)},
            "algo": {"num_algo": int(self.num_algo), "total_loop": int(self.total_loop)},
            "curves": {"cross": [float(x) for x in self.ep_reward_cross],
                       "wait": [float(x) for x in self.ep_reward_wait],
                       "choice": [float(x) for x in self.ep_reward_choice],
                       "balance": [[int(a), int(b)] for a, b in self.ep_scenario_balance]},
        }
        torch.save(ck, _rank_path(path))

    def load_checkpoint(self, path):
        """Inverse of save_checkpoint (weights_only load: tensors and plain containers only)."""
        ck = torch.load(_rank_path(path), map_location="cpu", weights_only=True)
        for name, sd in ck["nets"].items():
            k, h = name.split("_")
            getattr(self, f"{k}_net_{h}").load_state_dict(sd)
        for name, o in self._optimizers().items():
            o.load_state_dict(ck["optim"][name])
        self.venv.load_state_dict(ck["env"])
        self.rollout.iteration = ck["rollout"]["iteration"]
        self.rollout.seed = ck["rollout"]["seed"]
        self.num_algo, self.total_loop = ck["algo"]["num_algo"], ck["algo"]["total_loop"]
        c = ck["curves"]
        self.ep_reward_cross, self.ep_reward_wait = list(c["cross"]), list(c["wait"])
        self.ep_reward_choice, self.ep_scenario_balance = list(c["choice"]), [list(x) for x in c["balance"]]

    def saving(self):
        """(:985-1001)"""
        os.makedirs("load_model/weights", exist_ok=True)
        for head in ("cross", "wait", "choice"):
            for kind in ("actor", "critic"):
                net = getattr(self, f"{kind}_net_{head}")
                torch.save(net.state_dict(), self._path(head, kind, self.num_algo, self.total_loop))
