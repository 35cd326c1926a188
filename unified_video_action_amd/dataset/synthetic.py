"""Synthetic datasets in the reference datasets' sample layout (SURVEY §8(b) batch contract;
the zarr / LIBERO / UMI loaders themselves are out of scope).  Used by the shipped
configs (`task.dataset._target_`) for benchmarks and smoke runs; a reference dataset class can
be named instead when its package is importable.

One sample (CPU tensors, collated by torch's DataLoader):
  pusht:     obs.image [T,3,96,96] U[0,1], obs.agent_pos [T,2] U[0,512], action [T,2] U[0,512]
  libero_10: obs.agentview_rgb [T,3,128,128], action [T,10] U[-1,1], language_latents [512]
  umi:       obs.camera0_rgb [8,3,224,224], obs.robot0_* [T,d] N(0,1), obs.img_indices [8,1]
             (4 sorted history indices < 16, then 19,23,27,31 -- umi_lazy_dataset.py:271-285),
             action [T,10] N(0,1), language_latents [512]
Each sample is a pure function of (seed, index).
"""
import torch

from ..model.common.normalizer import LinearNormalizer

_TASKS = {
    "pusht": dict(key="image", frames=None, size=96, action_dim=2),
    "libero": dict(key="agentview_rgb", frames=None, size=128, action_dim=10),
    "umi": dict(key="camera0_rgb", frames=8, size=224, action_dim=10),
}


def _kind(task_name):
    for k in ("libero", "umi"):
        if k in task_name:
            return k
    return "pusht"


class SyntheticDataset(torch.utils.data.Dataset):
    def __init__(self, task_name="pusht", horizon=32, n_samples=512, seed=42, image_size=None, action_dim=None,
                 language_emb_model=None, normalizer_type="all", val_ratio=0.02, **kwargs):
        self.task_name = task_name
        self.kind = _kind(task_name)
        spec = _TASKS[self.kind]
        self.horizon = horizon
        self.n_samples = int(n_samples)
        self.seed = int(seed)
        self.key = spec["key"]
        self.frames = spec["frames"] or horizon
        self.size = image_size or spec["size"]
        self.action_dim = action_dim or spec["action_dim"]
        self.language_emb_model = language_emb_model
        self.normalizer_type = normalizer_type
        self.val_ratio = val_ratio

    def __len__(self):
        return self.n_samples

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + int(idx))
        T = self.horizon
        obs = {self.key: torch.rand(self.frames, 3, self.size, self.size, generator=g)}
        out = {"obs": obs}
        if self.kind == "pusht":
            obs["agent_pos"] = torch.rand(T, 2, generator=g) * 512
            out["action"] = torch.rand(T, self.action_dim, generator=g) * 512
        elif self.kind == "libero":
            out["action"] = torch.rand(T, self.action_dim, generator=g) * 2 - 1
        else:
            for k, d in (("robot0_eef_pos", 3), ("robot0_eef_rot_axis_angle", 6), ("robot0_gripper_width", 1),
                         ("robot0_eef_rot_axis_angle_wrt_start", 6)):
                obs[k] = torch.randn(T, d, generator=g)
            hist = torch.sort(torch.randperm(16, generator=g)[:4]).values
            obs["img_indices"] = torch.cat([hist, torch.tensor([19, 23, 27, 31])])[:, None].float()
            out["action"] = torch.randn(T, self.action_dim, generator=g)
        if self.language_emb_model is not None:
            out["language_latents"] = torch.randn(512, generator=g) * 0.1
        return out

    def get_validation_dataset(self):
        n = max(1, int(round(self.n_samples * self.val_ratio)))
        return SyntheticDataset(self.task_name, self.horizon, n, self.seed + 1, self.size, self.action_dim,
                                self.language_emb_model, self.normalizer_type, self.val_ratio)

    def get_normalizer(self, **kwargs):
        """"limits" fit over the sampling ranges (what fitting the full synthetic set converges to)."""
        n = LinearNormalizer()
        if self.kind == "pusht":
            lim = torch.tensor([[0.0] * self.action_dim, [512.0] * self.action_dim])
            n.fit({"action": lim, "agent_pos": lim[:, :2].clone()})
        elif self.kind == "libero":
            n.fit({"action": torch.tensor([[-1.0] * self.action_dim, [1.0] * self.action_dim])})
        return n
