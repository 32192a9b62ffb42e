"""GPU: nconv_amd.data.DevicePrefetcher delivers every batch of a DataLoader in HBM, unchanged and
in order, with the host-to-device copies on a side stream ordered before the consumer's use."""
import pytest
import torch
from torch.utils.data import DataLoader, TensorDataset

pytestmark = pytest.mark.gpu


def test_device_prefetcher_batches(nconv_amd, gpu):
    g = torch.Generator().manual_seed(0)
    depth = torch.rand(10, 1, 64, 96, generator=g)
    gt = torch.rand(10, 1, 64, 96, generator=g)

    class DS(TensorDataset):
        def __getitem__(self, i):
            d, t = super().__getitem__(i)
            return {"depth": d, "gt": t, "name": f"f{i}"}

    loader = DataLoader(DS(depth, gt), batch_size=4, pin_memory=True)
    seen = []
    for b in nconv_amd.data.DevicePrefetcher(loader, gpu):
        assert b["depth"].device.type == "cuda" and b["gt"].device.type == "cuda"
        seen.append((b["depth"] * 2).cpu())  # consumed on the compute stream
        assert isinstance(b["name"], list)
    torch.testing.assert_close(torch.cat(seen), depth * 2)
