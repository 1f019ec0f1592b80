# Import stub used ONLY by tools/gen_goldens.py to import the reference utils.py on CPU.
# fastbook is not installed in this image; utils.py only needs the names below from
# `from fastbook import *` (utils.py:1-2).  No arithmetic lives here.
import os, random
from pathlib import Path
import numpy as np
import torch
from torch import Tensor
from torch.nn import Module
