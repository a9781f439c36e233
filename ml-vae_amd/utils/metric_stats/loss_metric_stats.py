"""Per-batch loss log (ref:src/utils/metric_stats/loss_metric_stats.py:4-28).  Values are kept
as device tensors and read once at summarize(), not synchronised per batch."""
import torch


class LossMetricStats:
    def __init__(self, name):
        self.name = name
        self.clear()

    def clear(self):
        self.loss_list = []

    def append(self, loss):
        self.loss_list.append(loss.detach().reshape(()).clone())

    def summarize(self, field=None):
        if field is not None:
            raise ValueError('field must be None')
        if not self.loss_list:
            return {'loss': float('nan')}
        vals = torch.stack([v.to('cpu', torch.float32) for v in self.loss_list])
        return {'loss': vals.mean().item()}

    def write_stats(self, f):
        f.write(f'{self.name}: {self.summarize()}\n')
