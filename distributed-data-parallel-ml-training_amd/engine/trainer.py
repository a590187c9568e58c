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
import torch.nn as nn

from ..utils.misc import fault_point
from ..utils.trace import trace_range


class CrossEntropyLoss(nn.Module):
    """``nn.CrossEntropyLoss()`` (mean); GPU logits use the fused softmax-CE HIP kernel."""

    def forward(self, logits, target):
        if logits.is_cuda:
            from ..ops.layers import cross_entropy
            return cross_entropy(logits, target)
        return nn.functional.cross_entropy(logits, target)


def train_model(model, train_loader, optimizer, criterion, epoch, device="cpu", sync=None,
                log=print, metrics=None, watchdog=None, rank=0):
    running_loss = 0.0
    total_time = 0
    stats = {"iter_ns": []}
    for batch_idx, (data, target) in enumerate(train_loader):
        fault_point(rank, batch_idx)
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


def train_model_graph(step, train_loader, epoch, log=print, metrics=None, watchdog=None, rank=0):
    """``train_model`` over a captured TrainStep (engine/step.py): every iteration is ONE graph
    replay (augment + forward + backward + sync + optimizer) followed by a device synchronize,
    so the per-iteration timer keeps the reference's meaning (the reference's ``loss.item()``
    synchronises each iteration too). The loss print every 20 batches reads the device loss
    accumulator (same running mean as the reference).

    The captured step has a fixed batch shape, so only the floor(L/B) FULL batches of the shard
    are replays; a partial last batch (L % B samples, e.g. 80 of 50 000 at B = 256) runs as one
    eager step on exactly those samples (``TrainStep.tail_step``) — the same samples and the
    same partial-batch mean as the eager loop and the reference's DataLoader."""
    total_time = 0
    stats = {"iter_ns": []}
    nb = len(train_loader)
    L, B = train_loader.idx.numel(), train_loader.batch_size
    nfull = L // B
    step.pop_loss()
    for batch_idx in range(nb):
        fault_point(rank, batch_idx)
        start_time = time.perf_counter_ns()
        if batch_idx < nfull:
            step.step()
        else:
            step.tail_step(*train_loader.batch(batch_idx * B, L - batch_idx * B))
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
    if hasattr(step, "check_error"):
        step.check_error()
    stats["total_1_39_ns"] = total_time
    stats["graph_replays"] = min(nb, nfull)
    return stats


def graph_epoch_plan(n_samples, batch_size, max_batches=None):
    """(replayed full batches, eager tail size) of one --graph epoch over a shard of
    ``n_samples`` — the CPU-checkable schedule ``train_model_graph`` follows."""
    nb = -(-n_samples // batch_size)
    if max_batches:
        nb = min(nb, max_batches)
    nfull = min(nb, n_samples // batch_size)
    tail = n_samples - nfull * batch_size if nb > nfull else 0
    return nfull, tail


def test_model(model, test_loader, criterion, device="cpu", log=print, watchdog=None):
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
            if watchdog is not None:
                watchdog.beat()
    if fused:
        test_loss, correct = float(loss_acc), int(hits)
    n = len(test_loader.dataset)
    test_loss = float(test_loss) / max(nb, 1)
    log('Test set: Average loss: {:.4f}, Accuracy: {}/{} ({:.0f}%)\n'.format(
        test_loss, correct, n, 100. * correct / n))
    model.train()
    return test_loss, correct
