"""Pinned-memory H2D prefetch (utils/prefetch.py; SURVEY §8f-3, workspace:279-283 dict_apply .to)."""
import pytest
import torch

from unified_video_action_amd.utils.prefetch import PinnedPrefetcher


def _batches(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [{"obs": {"image": torch.rand(2, 4, 3, 8, 8, generator=g), "agent_pos": torch.rand(2, 4, 2, generator=g)},
             "action": torch.rand(2, 4, 2, generator=g), "dataset_name": f"d{i}", "idx": [torch.tensor(i)]}
            for i in range(n)]


def test_prefetch_cpu_identity_structure_and_order():
    src = _batches(5)
    got = list(PinnedPrefetcher(src, "cpu", depth=2))
    assert len(got) == 5 and len(PinnedPrefetcher(src, "cpu")) == 5
    for a, b in zip(got, src):
        assert a["dataset_name"] == b["dataset_name"] and isinstance(a["idx"], list)
        assert torch.equal(a["obs"]["image"], b["obs"]["image"]) and torch.equal(a["action"], b["action"])
    with pytest.raises(ValueError):
        PinnedPrefetcher(src, "cpu", depth=0)


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [1, 2, 3])
def test_prefetch_gpu_values_order_and_host_reuse(depth):
    """device batches equal the host batches in order; a loader that overwrites ONE host tensor in
    place for every batch (the copy must be staged before the next overwrite) still yields each
    batch's own values; a consumer kernel between batches does not disturb in-flight copies."""
    src = _batches(6, seed=1)
    shared = torch.empty_like(src[0]["obs"]["image"])

    def loader():
        for b in src:
            shared.copy_(b["obs"]["image"])  # same host storage every time
            yield {"obs": {"image": shared, "agent_pos": b["obs"]["agent_pos"]}, "action": b["action"],
                   "dataset_name": b["dataset_name"], "idx": b["idx"]}

    pf = PinnedPrefetcher(loader(), "cuda", depth=depth)
    for want, got in zip(src, pf):
        assert got["obs"]["image"].is_cuda and got["dataset_name"] == want["dataset_name"]
        torch.matmul(torch.rand(512, 512, device="cuda"), torch.rand(512, 512, device="cuda"))
        assert torch.equal(got["obs"]["image"].cpu(), want["obs"]["image"])
        assert torch.equal(got["action"].cpu(), want["action"]) and torch.equal(got["idx"][0].cpu(), want["idx"][0])
    assert pf.bytes_copied == sum(t.numel() * 4 for b in src for t in (b["obs"]["image"], b["obs"]["agent_pos"],
                                                                      b["action"])) + 6 * 8
