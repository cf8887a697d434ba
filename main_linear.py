"""Linear-probe evaluation entry point — CLI-compatible with the reference main_linear.py.

python main_linear.py --learning_rate 5 --batch_size 256 --ckpt path/to/last.pth
"""
from simclr_pytorch_distributed_amd.config import parse_linear
from simclr_pytorch_distributed_amd.engine.linear import LinearEngine
from simclr_pytorch_distributed_amd.utils.faults import guarded_main


def main(argv=None):
    opt = parse_linear(argv)
    return LinearEngine(opt).run()


if __name__ == "__main__":
    guarded_main(main)
