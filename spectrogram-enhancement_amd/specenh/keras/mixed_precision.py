"""keras.mixed_precision subset: the compute dtype of the conv kernels.

"float32" (Keras' default) runs the MFMA f32 path; "mixed_bfloat16" / "mixed_float16"
run bf16 / fp16 MFMA operands and activations with fp32 accumulation, fp32 master
weights, fp32 Adam state and fp32 logits for the loss (C4 trains in bf16, C5 infers in
fp16, SURVEY.md §8 d). Keras' loss scaling for mixed_float16 is not applied.
"""
_POLICIES = ("float32", "mixed_bfloat16", "mixed_float16")
_global = "float32"


class Policy:
    def __init__(self, name):
        if name not in _POLICIES:
            raise ValueError(f"policy {name!r} not supported (choose from {_POLICIES})")
        self.name = name

    @property
    def compute_dtype(self):
        return {"mixed_bfloat16": "bfloat16", "mixed_float16": "float16"}.get(self.name, "float32")

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
