"""Pinned-memory host->device batch prefetch (keep the GPUs fed).

The reference moves each dataloader batch with `dict_apply(batch, lambda x: x.to(device,
non_blocking=True))` on the compute stream right before the step
(workspace/train_unified_video_action_workspace.py:279-283, DataLoader pin_memory=True from
config/uva_pusht.yaml dataloader), so the copy of batch i+1 cannot start before step i's kernels
are queued behind it.  Here the copy runs on its own HIP stream, `depth` batches ahead:

* each batch's tensors are staged into a slot of page-locked host buffers (skipped for tensors the
  DataLoader already pinned), then copied by DMA on the copy stream; an event marks completion;
* a slot is refilled only after its previous copy's event has completed, so a loader that reuses
  its host tensors (or a caller that mutates them) never races the DMA;
* the consumer's stream waits on the event (no host sync) and the device tensors are tied to the
  consumer stream for the caching allocator (`record_stream`).

Nested dicts / lists / tuples are preserved; non-tensor leaves (e.g. `dataset_name`) pass through.
On a CPU device the prefetcher is the identity (there is no copy to overlap).
"""
import torch


def _map(x, fn):
    if isinstance(x, dict):
        return {k: _map(v, fn) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_map(v, fn) for v in x)
    return fn(x) if torch.is_tensor(x) else x


def _leaves(x, out):
    if isinstance(x, dict):
        for v in x.values():
            _leaves(v, out)
    elif isinstance(x, (list, tuple)):
        for v in x:
            _leaves(v, out)
    elif torch.is_tensor(x):
        out.append(x)
    return out


class _Slot:
    def __init__(self):
        self.bufs = []      # pinned staging tensors, one per leaf (reused while shapes match)
        self.event = None   # completion of this slot's last DMA


class PinnedPrefetcher:
    """Iterate `loader` with every batch already on `device`, copied `depth` batches ahead."""

    def __init__(self, loader, device, depth=2):
        if depth < 1:
            raise ValueError("depth must be >= 1")
        self.loader = loader
        self.device = torch.device(device)
        self.depth = depth
        self.cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(device=self.device) if self.cuda else None
        self.slots = [_Slot() for _ in range(depth)]
        self.bytes_copied = 0

    def __len__(self):
        return len(self.loader)

    def _stage(self, batch, slot):
        """host batch -> (device batch, event) with the DMA queued on the copy stream."""
        if slot.event is not None:
            slot.event.synchronize()  # the slot's previous DMA has read its pinned buffers
        leaves = _leaves(batch, [])
        if len(slot.bufs) != len(leaves) or any(b.shape != t.shape or b.dtype != t.dtype
                                                for b, t in zip(slot.bufs, leaves)):
            slot.bufs = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in leaves]
        it = iter(range(len(leaves)))

        def to_dev(t):
            i = next(it)
            if t.device.type != "cpu":
                return t.to(self.device, non_blocking=True)
            src = t if t.is_pinned() else slot.bufs[i].copy_(t)
            self.bytes_copied += t.numel() * t.element_size()
            return src.to(self.device, non_blocking=True)

        with torch.cuda.stream(self.stream):
            dev = _map(batch, to_dev)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        slot.event = ev
        return dev, ev

    def __iter__(self):
        if not self.cuda:
            yield from (_map(b, lambda t: t.to(self.device)) for b in self.loader)
            return
        src = iter(self.loader)
        queue = []
        k = 0
        for _ in range(self.depth):
            b = next(src, None)
            if b is None:
                break
            queue.append(self._stage(b, self.slots[k % self.depth]))
            k += 1
        cur = torch.cuda.current_stream(self.device)
        while queue:
            dev, ev = queue.pop(0)
            cur.wait_event(ev)
            for t in _leaves(dev, []):
                t.record_stream(cur)
            nxt = next(src, None)
            if nxt is not None:
                queue.append(self._stage(nxt, self.slots[k % self.depth]))
                k += 1
            yield dev
