"""Per-step bf16 weight cache for the native convolutions (and the projection head's
Linear layers, treated as 1x1 convs).

The fp32 master conv weights live in the flat parameter buffer (optim/flat.py) in
channels_last (KRSC) layout. Once per step, ONE kernel (csrc/kernels/wprep.hip) writes
every conv weight into a flat bf16 buffer in the two layouts the implicit-GEMM kernels
read: forward ``[K][R][S][Cp]`` (input channels zero-padded, e.g. 3→8 for the stem) and
data-gradient ``[C][R][S][K]``. Without a flat master buffer (e.g. a plain module on the
linear-probe path) the same layouts are produced per conv with torch ops.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch

from . import _ext


class ConvWeightCache:
    def __init__(self, convs: List[torch.nn.Conv2d], master: Optional[torch.Tensor] = None,
                 cin_pad: Optional[Dict[int, int]] = None):
        """``convs``: conv modules in any order; ``master``: flat fp32 buffer holding all
        their weights (channels_last), or None; ``cin_pad``: id(conv) -> padded Cin."""
        self.convs = convs
        self.master = master
        self.cin_pad = cin_pad or {}
        dev = convs[0].weight.device
        self.entries = {}
        rows = []
        off = 0
        tile0 = 0                             # first 64x64-tap tile of the next conv (wprep grid)
        ok = master is not None
        for cv in convs:
            w = cv.weight
            # nn.Linear [out][in] = a 1x1 conv: fwd layout W, dgrad layout Wᵀ
            K, C, R, S = w.shape if w.dim() == 4 else (w.shape[0], w.shape[1], 1, 1)
            Cp = self.cin_pad.get(id(cv), C)
            n_k = K * R * S * Cp
            want_t = Cp == C
            n_t = K * R * S * C if want_t else 0
            e = {"K": K, "C": C, "R": R, "S": S, "Cp": Cp, "off_k": off, "off_t": off + n_k if want_t else -1}
            off += n_k + n_t
            off = (off + 7) // 8 * 8          # keep every slice 16-byte aligned
            self.entries[id(cv)] = e
            if ok:
                if not (w.is_contiguous(memory_format=torch.channels_last) or (R == 1 and S == 1 and w.is_contiguous())):
                    ok = False
                else:
                    src = (w.data_ptr() - master.data_ptr()) // 4
                    if src < 0 or src + w.numel() > master.numel():
                        ok = False
                    rows.append([src, e["off_k"], e["off_t"], K | ((R * S) << 32), C | (Cp << 32), n_k, tile0])
                    tile0 += ((K + 63) // 64) * ((Cp + 63) // 64) * R * S
        self.tiles = tile0                    # wprep launches one block per tile
        self.seg_rows = rows                  # [src, off_k, off_t, K|RS<<32, C|Cp<<32, n_k, first tile]
        self.buf = torch.empty(off, dtype=torch.bfloat16, device=dev)
        self.native = ok and dev.type == "cuda" and _ext.available()
        self.segs = torch.tensor(rows, dtype=torch.int64, device=dev) if self.native else None
        self.version = -1
        self._pending = None     # event of a prefetch() issued on the side stream

    def prefetch(self):
        """Issue the next :meth:`refresh` now on the side stream (after all work queued so far
        on the current stream, i.e. the previous step's optimizer update), so the conversion
        overlaps the step's augmentation launch; :meth:`refresh` then only waits for it.
        Nothing the step reads before the first convolution depends on these weights."""
        from . import streams
        if not (self.native and streams.ENABLED):
            return
        dev = self.buf.device
        main = torch.cuda.current_stream(dev)
        s = streams.side(dev)
        s.wait_stream(main)
        with torch.cuda.stream(s):
            _ext.require().wprep(self.master, self.buf, self.segs, self.tiles)
        if getattr(self, "_ev", None) is None:
            self._ev = torch.cuda.Event()
        self._ev.record(s)
        self._pending = self._ev

    def refresh(self):
        """Re-derive all bf16 copies from the current fp32 master weights (one launch), or
        wait for the copy a :meth:`prefetch` already issued."""
        if self._pending is not None:
            torch.cuda.current_stream(self.buf.device).wait_event(self._pending)
            self._pending = None
            return
        if self.native:
            _ext.require().wprep(self.master, self.buf, self.segs, self.tiles)
        else:
            for cv in self.convs:
                e = self.entries[id(cv)]
                w = cv.weight.detach()
                w = w.view(w.shape[0], w.shape[1], 1, 1) if w.dim() == 2 else w
                w = w.permute(0, 2, 3, 1).to(torch.bfloat16)     # K R S C
                fk = self.fwd(cv)
                fk.zero_()
                fk[..., : e["C"]].copy_(w)
                if e["off_t"] >= 0:
                    self.dgrad(cv).copy_(w.permute(3, 1, 2, 0))

    def fwd(self, cv) -> torch.Tensor:
        e = self.entries[id(cv)]
        n = e["K"] * e["R"] * e["S"] * e["Cp"]
        return self.buf[e["off_k"]:e["off_k"] + n].view(e["K"], e["R"], e["S"], e["Cp"])

    def dgrad(self, cv) -> torch.Tensor:
        e = self.entries[id(cv)]
        n = e["K"] * e["R"] * e["S"] * e["C"]
        return self.buf[e["off_t"]:e["off_t"] + n].view(e["C"], e["R"], e["S"], e["K"])
