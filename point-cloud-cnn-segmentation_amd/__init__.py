"""pcs_amd — MI355X-native training hot path of seokjuchung/point-cloud-cnn-segmentation.

The drop-in boundary is ``pcs_amd.PointNetSegmentation`` (same constructor, forward
signature and 65-key state dict as the reference's ``PointNetSegmentation``,
point_cloud_segmentation.py:65-133).  Its compute runs in hand-written HIP kernels for
gfx950 behind a C-ABI library (``include/pcs.h``); there is no CPU fallback: using the
model on a device without the library raises.

Submodules are imported lazily so host-only pieces (``pcs_amd.data``) work on machines
without a GPU.
"""
__version__ = "0.1.0"

_LAZY = {
    "PointNetSegmentation": ("model", "PointNetSegmentation"),
    "FusedTrainStep": ("train", "FusedTrainStep"),
    "FusedAdam": ("optim", "FusedAdam"),
    "collate_fn": ("data", "collate_fn"),
    "load_reference_checkpoint": ("model", "load_reference_checkpoint"),
    "save_checkpoint": ("checkpoint", "save_checkpoint"),
    "load_checkpoint": ("checkpoint", "load_checkpoint"),
    "predict": ("checkpoint", "predict"),
    "ConfusionMeter": ("metrics", "ConfusionMeter"),
    "RaggedBatch": ("data", "RaggedBatch"),
    "ragged_collate": ("data", "ragged_collate"),
    "CSRPointCloudDataset": ("data", "CSRPointCloudDataset"),
    "PointCloudDataset": ("data", "PointCloudDataset"),
    "pad_on_device": ("loader", "pad_on_device"),
    "DevicePrefetcher": ("loader", "DevicePrefetcher"),
    "voxelize": ("voxel", "voxelize"),
    "voxel_ids": ("voxel", "voxel_ids"),
}


def __getattr__(name):
    if name in _LAZY:
        import importlib
        mod, attr = _LAZY[name]
        return getattr(importlib.import_module(f"{__name__}.{mod}"), attr)
    if name in ("data", "model", "optim", "train", "engine", "metrics", "checkpoint", "loader", "voxel"):
        import importlib
        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)
