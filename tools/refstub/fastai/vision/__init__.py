# Import stub for tools/gen_goldens.py (`from fastai.vision import *`, utils.py:501).
