"""Model_PPO — the reference's multi-head MLP (Coop-MH-PPO-scalable.py:42-93).

Same constructor signature, same submodule names (`layer1..layer4`, so shipped
`.pth` state_dicts load), same construction order (so `torch.manual_seed(s)`
yields the reference's initial weights), same forward.  `packed()` lays the
weights out contiguously for the HIP rollout kernels (include/mhppo.h mhppo_mlp).
"""
import ctypes

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib


class Model_PPO(nn.Module):
    """in -> 32 -> 64 -> 32 -> out, ReLU.  model_type 2: pairwise softmax (choice actor);
    1: tanh * std + mean (continuous actor); 0: linear (critics)."""

    def __init__(self, np_inputs, nb_outputs, model_type=0, nb_car=1, mean=0, std=1):
        super().__init__()
        self.model_type = model_type
        self.nb_car = nb_car
        self.mean = mean
        self.std = std
        self.layer1 = nn.Linear(np_inputs, 32)
        self.layer2 = nn.Linear(32, 64)
        self.layer3 = nn.Linear(64, 32)
        self.layer4 = nn.Linear(32, nb_outputs)
        # The reference re-creates layer4 for types 2 and 1 (:58-64): keep that RNG use.
        if self.model_type == 2:
            self.layer4 = nn.Linear(32, nb_outputs)
            self.return_layer = nn.Softmax(dim=-1)
        if self.model_type == 1:
            self.layer4 = nn.Linear(32, nb_outputs)
            self.return_layer = nn.Tanh()
        torch.nn.init.orthogonal_(self.layer4.weight)
        self._flatten()

    # ---- flat storage: the parameters (and their .grad) are views of ONE contiguous
    # float32 vector in the packed torch layout W1 b1 W2 b2 W3 b3 W4 b4, so the HIP kernels
    # read the weights and write the gradient in place (no per-launch cat / copy), and one
    # fused Adam launch updates a whole net.
    def _params(self):
        # straight from the module / parameter dicts (nn.Module.__getattr__ costs ~1 us a lookup, and
        # flat() / grad_flat() run once per head and update): always the current registrations
        m = self._modules
        return [q for lay in (m["layer1"], m["layer2"], m["layer3"], m["layer4"])
                for q in (lay._parameters["weight"], lay._parameters["bias"])]

    def _flatten(self):
        ps = self._params()
        flat = torch.cat([p.detach().reshape(-1) for p in ps]).float().contiguous()
        gb = getattr(self, "_gbound", None)  # storage given by bind_grad (a GradBucket slice)
        if gb is not None and gb.numel() == flat.numel() and gb.device == flat.device:
            gflat = gb
        else:
            gflat = torch.zeros_like(flat)
        off = 0
        with torch.no_grad():
            for p in ps:
                n = p.numel()
                p.data = flat[off:off + n].view_as(p)
                p.grad = gflat[off:off + n].view_as(p)
                off += n
        self._flat, self._gflat = flat, gflat

    def _apply(self, fn, *args, **kwargs):
        super()._apply(fn, *args, **kwargs)  # .to()/.cuda() move each parameter: re-flatten
        self._flatten()
        return self

    def flat(self):
        """The live flat parameter vector (no copy); re-flattens if a parameter was rebound."""
        off = 0
        base = self._flat.data_ptr()
        for p in self._params():
            if p.data_ptr() != base + 4 * off or p.dtype != torch.float32:
                self._flatten()
                return self._flat
            off += p.numel()
        return self._flat

    def grad_flat(self):
        """The flat gradient vector the parameters' .grad views alias (re-linked if
        zero_grad(set_to_none=True) or autograd replaced a .grad)."""
        self.flat()
        off = 0
        base = self._gflat.data_ptr()
        for p in self._params():
            n = p.numel()
            if p.grad is None or p.grad.data_ptr() != base + 4 * off:
                if p.grad is not None:
                    self._gflat[off:off + n].copy_(p.grad.reshape(-1))
                p.grad = self._gflat[off:off + n].view_as(p)
            off += n
        return self._gflat

    def bind_grad(self, storage):
        """Make `storage` (float32, one element per parameter, on the net's device) the flat
        gradient the parameters' .grad views alias (mhppo.ppo.GradBucket)."""
        if storage.numel() != self.flat().numel() or storage.dtype != torch.float32:
            raise ValueError("gradient storage must be float32 with one element per parameter")
        self._gbound = storage
        self._gflat = storage
        off = 0
        with torch.no_grad():
            for p in self._params():
                n = p.numel()
                p.grad = storage[off:off + n].view_as(p)
                off += n
        return self

    def forward(self, input1):
        if isinstance(input1, np.ndarray):
            input1 = torch.tensor(input1, dtype=torch.float, device=self.layer1.weight.device)
        a1 = F.relu(self.layer1(input1))
        a2 = F.relu(self.layer2(a1))
        a3 = F.relu(self.layer3(a2))
        if self.model_type == 2:
            out = self.layer4(a3).reshape(-1, 2)
            return torch.flatten(self.return_layer(out))
        if self.model_type == 1:
            out = self.layer4(a3)
            return torch.add(torch.mul(self.return_layer(out), self.std), self.mean)
        return self.layer4(a3)

    @property
    def n_in(self):
        return self.layer1.in_features

    @property
    def n_out(self):
        return self.layer4.out_features

    def packed(self):
        """Contiguous float32 copy W1 b1 W2 b2 W3 b3 W4 b4 (torch layouts) on the model's device."""
        parts = []
        for lay in (self.layer1, self.layer2, self.layer3, self.layer4):
            parts += [lay.weight.detach().reshape(-1), lay.bias.detach().reshape(-1)]
        return torch.cat(parts).float().contiguous()

    def load_packed(self, flat):
        """Inverse of packed(): load a flat W1 b1 .. W4 b4 vector into the layers."""
        flat = torch.as_tensor(flat, dtype=torch.float32).reshape(-1)
        off = 0
        with torch.no_grad():
            for lay in (self.layer1, self.layer2, self.layer3, self.layer4):
                for p in (lay.weight, lay.bias):
                    n = p.numel()
                    p.copy_(flat[off:off + n].view_as(p))
                    off += n
        if off != flat.numel():
            raise ValueError(f"packed size {flat.numel()} != model size {off}")
        return self

    def mlp_desc(self, packed=None):
        """(mhppo_mlp struct, backing tensor) for the C-ABI (the live flat weights)."""
        t = self.flat() if packed is None else packed
        d = _lib.Mlp()
        d.packed = ctypes.c_void_p(t.data_ptr())
        d.n_in, d.n_out = self.n_in, self.n_out
        d.kind = self.model_type
        d.mean = float(self.mean)
        d.std = float(self.std)
        return d, t
