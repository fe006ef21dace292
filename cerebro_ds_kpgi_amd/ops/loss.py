"""Fused softmax cross-entropy + top-1/top-5 metrics for G packed configs.

logits ``[B, G*N]`` (config g owns columns ``g*N:(g+1)*N``), labels
``[G, B]`` int32.  Per config: mean CE over the batch (= Keras
``categorical_crossentropy`` / torch ``CrossEntropyLoss``), and the metric
accumulator ``acc[g] += (loss_sum, top1_correct, top5_correct, count)``
on device — no host sync per step (reference metrics: SURVEY.md §5.5,
``cerebro_gpdb/run_pytorchddp.py:181-201``).  For N == 2 (Criteo) top-5 is
reported as 1 (reference binary-accuracy path).
"""

import torch

from .backend import use_hip


class SoftmaxCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, acc, G, head=None, unit=False):
        B = logits.shape[0]
        N = logits.shape[1] // G
        ctx.unit = unit
        if unit and logits.dtype == torch.float32 and use_hip("loss", logits):
            # training step: the caller seeds a unit gradient and reads the
            # metrics from ``acc`` -- no loss values, and the head's bias
            # gradient comes out of this kernel (``head`` = (bias ref, box))
            from . import _hip
            dlogits = _hip.softmax_ce_train(logits, labels, acc, G,
                                            head[0] if head is not None else None)
            if head is not None:
                head[1][0] = True
            ctx.save_for_backward(dlogits)
            ctx.dtype = logits.dtype
            return logits.new_empty(G)
        if use_hip("loss", logits):
            from . import _hip
            loss, dlogits = _hip.softmax_ce_fwd(logits, labels, acc, G)
        else:
            z = logits.view(B, G, N).float()
            lse = torch.logsumexp(z, dim=2)                             # [B, G]
            lab = labels.t().long()                                     # [B, G]
            picked = z.gather(2, lab.unsqueeze(2)).squeeze(2)
            nll = lse - picked                                          # [B, G]
            loss = nll.mean(0)                                          # [G]
            p = torch.softmax(z, dim=2)
            onehot = torch.zeros_like(p).scatter_(2, lab.unsqueeze(2), 1.0)
            dlogits = ((p - onehot) / B).reshape(B, G * N)
            with torch.no_grad():
                k = min(5, N)
                top = z.topk(k, dim=2).indices                          # [B, G, k]
                hit = top == lab.unsqueeze(2)
                top1 = hit[:, :, 0].float().sum(0)
                top5 = hit.any(2).float().sum(0) if N > 2 else torch.full_like(top1, float(B))
                acc += torch.stack([nll.sum(0), top1, top5, torch.full_like(top1, float(B))], 1)
        ctx.save_for_backward(dlogits)
        ctx.dtype = logits.dtype
        return loss

    @staticmethod
    def backward(ctx, dloss):
        dlogits, = ctx.saved_tensors
        if ctx.unit:                    # dloss is ones by the caller's contract
            return dlogits.to(ctx.dtype), None, None, None, None, None
        B, GN = dlogits.shape
        G = dloss.shape[0]
        d = dlogits.view(B, G, GN // G) * dloss.view(1, G, 1)
        return d.reshape(B, GN).to(ctx.dtype), None, None, None, None, None


def softmax_ce(logits, labels, acc, G, head=None, unit=False):
    """Per-config mean CE ``[G]``.  ``unit=True``: the caller back-propagates
    a gradient of ones (``torch.autograd.backward(loss, ones)``), so the
    backward returns dlogits as they are; on the fp32 HIP path the returned
    loss values are then not computed (metrics live in ``acc``).  ``head``:
    ``logits._cer_head`` of an act-free Dense (ops.nn.PackedLinear) whose
    bias gradient the loss kernel then accumulates."""
    return SoftmaxCE.apply(logits, labels, acc, G, head, unit)


def eval_metrics(logits, labels, acc, G):
    """Validation: same accumulators, no gradient."""
    with torch.no_grad():
        if use_hip("loss", logits):
            from . import _hip
            _hip.softmax_ce_fwd(logits, labels, acc, G, need_grad=False)
            return
        SoftmaxCE.forward(_Ctx(), logits, labels, acc, G)


class _Ctx(object):
    def save_for_backward(self, *a):
        pass
