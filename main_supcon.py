"""Contrastive pretraining entry point (SimCLR / SupCon) — CLI-compatible with the
reference main_supcon.py (same flags, defaults, work_space layout, log format).

Single GPU:   python main_supcon.py --batch_size 256 --epochs 100 --cosine --temp 0.5
Multi GPU:    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 main_supcon.py --syncBN ...
              (python -m torch.distributed.launch ... --local_rank=N also accepted)
CPU:          python main_supcon.py --backend torch --dist_backend gloo --batch_size 16 ...
"""
from simclr_pytorch_distributed_amd.config import parse_pretrain
from simclr_pytorch_distributed_amd.engine.pretrain import PretrainEngine
from simclr_pytorch_distributed_amd.utils.faults import guarded_main


def main(argv=None):
    opt = parse_pretrain(argv)
    engine = PretrainEngine(opt)
    return engine.run()


if __name__ == "__main__":
    guarded_main(main)
