# Import stub for tools/gen_goldens.py (fastai is not installed; utils.py:501).
