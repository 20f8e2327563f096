"""Known-byte-count read probes for calibrating rocprofv3 FETCH_SIZE on gfx950
(MI355X_MICROARCH.md §HBM: calibrate on your own access pattern).  Run under
`rocprofv3 --pmc FETCH_SIZE`; each pattern is one dispatch over exactly BYTES bytes
(4 GiB: far past the 256 MiB Infinity Cache, so no re-read is absorbed on-die)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BYTES = 4 << 30


def main():
    import spacedrive_amd as sd
    from spacedrive_amd._native import check, lib
    ctx = sd.Context(0)
    buf = torch.ones(BYTES, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    for pattern in (0, 1, 2):
        check(lib().sd_read_probe(ctx.handle, buf.data_ptr(), BYTES, pattern, None))
        torch.cuda.synchronize()
    print({"bytes": BYTES, "patterns": [0, 1, 2]})


if __name__ == "__main__":
    main()
