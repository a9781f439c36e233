"""FileTrainLogger: one line per stage ("epoch: 1 - train loss: 1.2") appended to a file."""


def _fmt(stats):
    return ", ".join(f"{k}: {v:.3g}" if isinstance(v, float) else f"{k}: {v}" for k, v in stats.items())


class FileTrainLogger:
    def __init__(self, save_file, precision=2):
        self.save_file = str(save_file)
        self.precision = precision

    def log_stats(self, stats_meta, train_stats=None, valid_stats=None, test_stats=None,
                  verbose=False):
        parts = [_fmt(stats_meta)]
        for name, st in (("train", train_stats), ("valid", valid_stats), ("test", test_stats)):
            if st:
                parts.append(", ".join(f"{name} {k}: {v}" for k, v in st.items()))
        with open(self.save_file, "a") as f:
            f.write(" - ".join(parts) + "\n")
