"""tools/export_azw.py on a state_dict with the reference ResNet's key layout: header and blob
order match what HipNeuralNetwork::load expects (the canonical blob of oracle/net_oracle)."""
import os
import struct
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_export_azw_roundtrip(tmp_path):
    import torch
    import az_amd
    import net_oracle
    desc = az_amd.gomoku_net_desc(board_size=9, channels=16, blocks=2, max_batch=4)
    blob = net_oracle.init_blob(desc, seed=3)
    sd, off = {}, 0
    for name, shp, _, _ in net_oracle.param_shapes(desc):
        n = int(np.prod(shp))
        sd[name] = torch.from_numpy(blob[off:off + n].reshape(shp).copy())
        off += n
        if name.endswith("running_var"):
            sd[name[:-len("running_var")] + "num_batches_tracked"] = torch.tensor(0)
    src, dst = tmp_path / "m.pt", tmp_path / "m.azw"
    torch.save(sd, src)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "export_azw.py"), str(src), str(dst),
                    "--max-batch", "4"], check=True, capture_output=True)
    raw = dst.read_bytes()
    assert raw[:4] == b"AZW1"
    hdr = struct.unpack("<12i", raw[4:52])
    assert hdr == (9, 11, 16, 2, 81, 32, 8, 256, 1, 0, 3, 4)
    (count,) = struct.unpack("<Q", raw[52:60])
    assert count == blob.size and np.array_equal(np.frombuffer(raw[60:], np.float32), blob)
