"""keras.callbacks subset: History and EarlyStopping (manual_scan_3layers.py:25,172)."""
import numpy as np


class Callback:
    model = None

    def set_model(self, model):
        self.model = model

    def on_train_begin(self, logs=None):
        pass

    def on_epoch_end(self, epoch, logs=None):
        pass

    def on_train_end(self, logs=None):
        pass


class History(Callback):
    """fit()'s return value: .history['loss' | 'val_loss'] lists, .epoch, .params."""

    def __init__(self):
        self.history = {}
        self.epoch = []
        self.params = {}

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(v)


class EarlyStopping(Callback):
    def __init__(self, monitor="val_loss", min_delta=0, patience=0, verbose=0, mode="auto",
                 baseline=None, restore_best_weights=False, start_from_epoch=0):
        self.monitor, self.patience, self.verbose = monitor, patience, verbose
        self.baseline, self.restore_best_weights = baseline, restore_best_weights
        self.start_from_epoch = start_from_epoch
        if mode == "auto":
            mode = "max" if "acc" in monitor else "min"
        self.op = np.less if mode == "min" else np.greater
        self.min_delta = abs(min_delta) * (1 if mode == "max" else -1)
        self.stopped_epoch = 0

    def on_train_begin(self, logs=None):
        self.wait = 0
        self.stopped_epoch = 0
        self.best = np.inf if self.op is np.less else -np.inf
        self.best_weights = None
        self.best_epoch = 0

    def on_epoch_end(self, epoch, logs=None):
        current = (logs or {}).get(self.monitor)
        if current is None or epoch < self.start_from_epoch:
            return
        if self.restore_best_weights and self.best_weights is None:
            self.best_weights = self.model.get_weights()
        self.wait += 1
        if self.op(current - self.min_delta, self.best):
            self.best, self.best_epoch = current, epoch
            if self.restore_best_weights:
                self.best_weights = self.model.get_weights()
            if self.baseline is None or self.op(current - self.min_delta, self.baseline):
                self.wait = 0
        if self.wait >= self.patience and epoch > 0:
            self.stopped_epoch = epoch
            self.model.stop_training = True
            if self.restore_best_weights and self.best_weights is not None:
                self.model.set_weights(self.best_weights)

    def on_train_end(self, logs=None):
        if self.stopped_epoch > 0 and self.verbose > 0:
            print(f"Epoch {self.stopped_epoch + 1}: early stopping")
