"""Does torch's CPU inverse return the same bits for a stride-0 / F-ordered / sliced K on this
host as on the host that made tests/golden/kstride.npz?  Prints one JSON line per case."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "tests"))
from test_kstride import make_layout  # noqa: E402

ks = np.load(os.path.join(REPO, "tests", "golden", "kstride.npz"))
print(json.dumps({"torch": torch.__version__, "mkl": torch.backends.mkl.is_available(),
                  "threads": torch.get_num_threads(), "config": torch.__config__.show()[:2000]}))
for c in ("psv_expand", "psv_fortran", "psv_slice", "piw_expand"):
    K = torch.tensor(ks[c + "_K"])
    lay = str(ks[c + "_layout"])
    a = torch.inverse(make_layout(K, lay))
    b = torch.inverse(K.contiguous())
    print(json.dumps({"case": c, "layout_differs_from_contiguous": not torch.equal(a, b),
                      "bits": a.contiguous().numpy().view(np.uint32).reshape(-1)[:9].tolist(),
                      "bits_contig": b.contiguous().numpy().view(np.uint32).reshape(-1)[:9].tolist()}))
