"""simclr_pytorch_distributed_amd — MI355X-native SimCLR / SupCon pretraining framework.

Capabilities of Dyfine/SimCLR_pytorch_distributed (main_supcon.py / main_linear.py CLI,
checkpoint layout, SimCLR+SupCon losses, SyncBN + data parallel) re-designed for
AMD MI355X (gfx950): hand-written HIP/CDNA4 kernels for the hot ops, RCCL collectives
over xGMI, HIP streams/graphs around them.
"""
__version__ = "0.1.0"
