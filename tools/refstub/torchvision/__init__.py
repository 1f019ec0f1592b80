# Import stub for tools/gen_goldens.py; only show_torch_image (utils.py:507, out of scope) uses it.
class transforms:  # noqa: N801
    pass
