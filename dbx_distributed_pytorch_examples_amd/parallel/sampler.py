"""Rank partitioning of a dataset (the reference's ``DistributedSampler``).

Used at `/root/reference/01_torch_distributor/01_basic_torch_distributor.py:285-286` and via Ray's
``prepare_data_loader`` + ``sampler.set_epoch`` (`05_ray/01_fashion_mnist_pytorch_ray.ipynb:185-190`).
Semantics match torch's DistributedSampler (seed + epoch permutation, padding by wrap-around
or drop_last) so results are comparable; no communication is involved.
"""
from __future__ import annotations

import math
from typing import Iterator, Optional

import torch
from torch.utils.data import Sampler

from . import dist as ddist


class ShardSampler(Sampler[int]):
    def __init__(self, dataset_or_len, num_replicas: Optional[int] = None, rank: Optional[int] = None,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False):
        self.n = dataset_or_len if isinstance(dataset_or_len, int) else len(dataset_or_len)
        self.num_replicas = num_replicas if num_replicas is not None else ddist.get_world_size()
        self.rank = rank if rank is not None else ddist.get_rank()
        if not 0 <= self.rank < self.num_replicas:
            raise ValueError(f"rank {self.rank} out of range for world {self.num_replicas}")
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0
        if drop_last and self.n % self.num_replicas:
            self.num_samples = self.n // self.num_replicas
        else:
            self.num_samples = math.ceil(self.n / self.num_replicas)
        self.total_size = self.num_samples * self.num_replicas

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def indices(self) -> torch.Tensor:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g)
        else:
            idx = torch.arange(self.n)
        if not self.drop_last:
            pad = self.total_size - self.n
            if pad > 0:
                reps = math.ceil(pad / max(1, self.n))
                idx = torch.cat([idx] + [idx] * reps)[:self.total_size]
        else:
            idx = idx[:self.total_size]
        return idx[self.rank:self.total_size:self.num_replicas]

    def __iter__(self) -> Iterator[int]:
        return iter(self.indices().tolist())

    def __len__(self) -> int:
        return self.num_samples


# torch-compatible alias (the reference imports DistributedSampler by that name)
DistributedSampler = ShardSampler
