from collections import OrderedDict
import numpy as np


class Box:
    def __init__(self, low=None, high=None, shape=None, dtype=np.float32):
        self.low, self.high, self.dtype = low, high, dtype
        self.shape = tuple(shape) if shape is not None else np.shape(low)

    def sample(self):
        return np.zeros(self.shape, dtype=self.dtype)


class Discrete:
    def __init__(self, n):
        self.n = n


class Dict:
    def __init__(self, spaces):
        if isinstance(spaces, dict) and not isinstance(spaces, OrderedDict):
            spaces = OrderedDict(sorted(spaces.items()))
        self.spaces = OrderedDict(spaces)

    def __getitem__(self, k):
        return self.spaces[k]

    def sample(self):
        return OrderedDict((k, v.sample()) for k, v in self.spaces.items())
