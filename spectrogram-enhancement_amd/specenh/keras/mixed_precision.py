"""keras.mixed_precision subset: the compute dtype of the conv kernels.

"float32" (Keras' default) runs the MFMA f32 path; "mixed_bfloat16" runs bf16 MFMA
operands and activations with fp32 accumulation, fp32 master weights, fp32 Adam state
and fp32 logits for the loss (the C4 training configuration, SURVEY.md §8 d).
"""
_POLICIES = ("float32", "mixed_bfloat16")
_global = "float32"


class Policy:
    def __init__(self, name):
        if name not in _POLICIES:
            raise ValueError(f"policy {name!r} not supported (choose from {_POLICIES})")
        self.name = name

    @property
    def compute_dtype(self):
        return "bfloat16" if self.name == "mixed_bfloat16" else "float32"

    @property
    def variable_dtype(self):
        return "float32"

    def __repr__(self):
        return f'<Policy "{self.name}">'


def set_global_policy(policy):
    global _global
    _global = Policy(policy if isinstance(policy, str) else policy.name).name


def global_policy():
    return Policy(_global)
