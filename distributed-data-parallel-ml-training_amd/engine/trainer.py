"""Training and evaluation loops with the reference's observable behaviour.

Reference parity: ``train_model`` (part1/main.py:52-93; part2/part2a/main.py:118-160 with the
sync call at :143) and ``test_model`` (part1/main.py:96-111):
* per batch: timer start -> ``.to(device)`` -> zero_grad -> forward -> loss -> backward ->
  [gradient sync] -> step -> ``loss.item()``;
* ``[epoch, batch] loss: x.xxx`` every 20 batches (rank-local running mean, not all-reduced);
* iteration 0 is warm-up; the wall time of iterations 1..39 is summed and printed at 39;
* eval: model.eval(), no_grad, sum of per-batch mean CE divided by the NUMBER OF BATCHES,
  argmax accuracy over the whole (unsharded) test set, reference print format.
"""
import time

import torch

from ..utils.trace import trace_range
import torch.nn as nn


class CrossEntropyLoss(nn.Module):
    """``nn.CrossEntropyLoss()`` (mean); GPU logits use the fused softmax-CE HIP kernel."""

    def forward(self, logits, target):
        if logits.is_cuda:
            from ..ops.layers import cross_entropy
            return cross_entropy(logits, target)
        return nn.functional.cross_entropy(logits, target)


def train_model(model, train_loader, optimizer, criterion, epoch, device="cpu", sync=None,
                log=print, metrics=None, watchdog=None):
    running_loss = 0.0
    total_time = 0
    stats = {"iter_ns": []}
    for batch_idx, (data, target) in enumerate(train_loader):
        start_time = time.perf_counter_ns()
        with trace_range("data"):
            data, target = data.to(device), target.to(device)

        optimizer.zero_grad()
        with trace_range("forward"):
            output = model(data)
            loss = criterion(output, target)
        with trace_range("backward"):
            loss.backward()
        if sync is not None:
            with trace_range("sync"):
                sync(model)
        with trace_range("optimizer"):
            optimizer.step()

        running_loss += loss.item()
        if batch_idx % 20 == 19:
            log(f'[{epoch + 1}, {batch_idx + 1:5d}] loss: {running_loss / 20:.3f}')
            running_loss = 0.0

        dt = time.perf_counter_ns() - start_time
        stats["iter_ns"].append(dt)
        if 0 < batch_idx < 40:
            total_time += dt
        if batch_idx == 39:
            log(f'Total time for 1-39 iteration in ns: {total_time}')
            log(f'Average time for 1-39 iteration in ns: {total_time / 39.0}')
        if metrics is not None:
            metrics.log(event="iter", epoch=epoch, batch=batch_idx, ns=dt)
        if watchdog is not None:
            watchdog.beat()
    stats["total_1_39_ns"] = total_time
    return stats


def train_model_graph(step, train_loader, epoch, log=print, metrics=None, watchdog=None):
    """``train_model`` over a captured TrainStep (engine/step.py): every iteration is ONE graph
    replay (augment + forward + backward + sync + optimizer) followed by a device synchronize,
    so the per-iteration timer keeps the reference's meaning (the reference's ``loss.item()``
    synchronises each iteration too). The loss print every 20 batches reads the device loss
    accumulator (same running mean as the reference)."""
    total_time = 0
    stats = {"iter_ns": []}
    nb = len(train_loader)
    step.pop_loss()
    for batch_idx in range(nb):
        start_time = time.perf_counter_ns()
        step.step()
        torch.cuda.synchronize()
        if batch_idx % 20 == 19:
            log(f'[{epoch + 1}, {batch_idx + 1:5d}] loss: {step.pop_loss() / 20:.3f}')
        dt = time.perf_counter_ns() - start_time
        stats["iter_ns"].append(dt)
        if 0 < batch_idx < 40:
            total_time += dt
        if batch_idx == 39:
            log(f'Total time for 1-39 iteration in ns: {total_time}')
            log(f'Average time for 1-39 iteration in ns: {total_time / 39.0}')
        if metrics is not None:
            metrics.log(event="iter", epoch=epoch, batch=batch_idx, ns=dt)
        if watchdog is not None:
            watchdog.beat()
    stats["total_1_39_ns"] = total_time
    return stats


def test_model(model, test_loader, criterion, device="cpu", log=print):
    model.eval()
    test_loss = 0
    correct = 0
    nb = 0
    inner = getattr(model, "module", model)
    fused = (torch.device(device).type == "cuda" and hasattr(inner, "forward_metrics")
             and type(criterion) is CrossEntropyLoss)
    if fused:  # loss + argmax hits accumulated on the device by the classifier kernel
        loss_acc = torch.zeros((), dtype=torch.float32, device=device)
        hits = torch.zeros((), dtype=torch.int32, device=device)
    with torch.no_grad():
        for data, target in test_loader:
            data, target = data.to(device), target.to(device)
            if fused:
                inner.forward_metrics(data, target, loss_acc, hits)
            else:
                output = model(data)
                test_loss += criterion(output, target)
                pred = output.max(1, keepdim=True)[1]
                correct += pred.eq(target.view_as(pred)).sum().item()
            nb += 1
    if fused:
        test_loss, correct = float(loss_acc), int(hits)
    n = len(test_loader.dataset)
    test_loss = float(test_loss) / max(nb, 1)
    log('Test set: Average loss: {:.4f}, Accuracy: {}/{} ({:.0f}%)\n'.format(
        test_loss, correct, n, 100. * correct / n))
    model.train()
    return test_loss, correct
