"""CORAL domain loss (reference src/utils/coral_loss/coral.py:5-37): the squared
Frobenius distance between the two domains' second-moment matrices, / (4 d^2).

Reference quirk kept for parity: its "covariance" is (X^T X - mu^T mu) / (n - 1)
with mu the column mean (coral.py:31-35), i.e. the mean outer product is
subtracted once, not n times, so it is not the centred covariance.  Same value
and the same NaN for a one-sample domain (n - 1 = 0).  Runs on the features'
device; the mu^T mu correction is applied to X^T X as a
rank-1 addmm update.
"""
import torch


def compute_covariance(input_data: torch.Tensor) -> torch.Tensor:
    n = input_data.shape[0]
    mu = input_data.mean(dim=0, keepdim=True)
    return torch.addmm(input_data.t() @ input_data, mu.t(), mu, alpha=-1.0) / (n - 1)


def coral(source: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    d = source.shape[1]
    diff = compute_covariance(source) - compute_covariance(target)
    return (diff * diff).sum() / (4 * d * d)
