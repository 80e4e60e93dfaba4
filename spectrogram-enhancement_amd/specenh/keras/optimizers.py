"""keras.optimizers.Adam (Keras defaults; the form w -= lr_t m / (sqrt(v) + eps))."""


class Adam:
    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7,
                 amsgrad=False, name="Adam", **kwargs):
        if amsgrad:
            raise NotImplementedError("amsgrad")
        self.learning_rate = float(learning_rate)
        self.beta_1, self.beta_2, self.epsilon = float(beta_1), float(beta_2), float(epsilon)
        self.name = name

    def get_config(self):
        return {"name": self.name, "learning_rate": self.learning_rate, "beta_1": self.beta_1,
                "beta_2": self.beta_2, "epsilon": self.epsilon}


def get(identifier):
    if isinstance(identifier, Adam):
        return identifier
    if isinstance(identifier, str) and identifier.lower() == "adam":
        return Adam()
    raise NotImplementedError(f"optimizer {identifier!r}: only Adam is implemented")
