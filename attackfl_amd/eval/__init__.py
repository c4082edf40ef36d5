"""Server-side validation (reference ``src/Validation.py:19-214``).

ICU: ROC-AUC over the whole test set (``ROC_AUC: x.xxxx`` in ``app.log``); NaN outputs fail the
round.  HAR: accuracy.  CIFAR10 (``test_image`` / ``test_hyper_image``, ``src/Validation.py:69-90,
147-175``): summed NLL of the model's log-probabilities over the test set divided by its length, and
``100 * correct / len`` accuracy; a NaN or ``|loss| > 1e6`` fails the round.  The hyper variant
pools every client's loss and hits but still divides by ONE test-set length, like the reference.  ``test_hyper`` pools the outputs of every client's hypernetwork-generated
model before one ROC-AUC, like ``test_hyper_icu``.  The test set stays resident on the device
and is evaluated in one pass (eval mode is batch-size independent).  On GPU every ICU / HAR model
runs a native forward: TransformerModel / RNNModel / CNNModel their fused HIP eval kernels (C models per launch),
TransformerClassifier its layer program (``fl/programs.py``) in eval mode.  CIFAR10 images (the
reference ships no image model) go through the eager PyTorch module on either device.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

from .. import ops
from ..data import DeviceTable, HARData, ICUData, resolve_dataset
from ..models import ParamLayout, build_model
from ..utils.log import print_with_color

EVAL_CHUNK = 65536
PROGRAM_EVAL_BATCH = {"CNNModel": 4096, "RNNModel": 16384, "TransformerClassifier": 256}


def cnn_eval_many(params: torch.Tensor, rows: torch.Tensor, layout: Optional[ParamLayout] = None) -> torch.Tensor:
    """Sigmoid outputs of C CNNModels (``params [C, P]``, eval mode) over ICU ``rows [n, 24]`` -> ``[C, n]``: one
    launch (``cnn2.hip`` ``k_cnn2_eval``: bf16 MFMA convolutions and fc1, fp32 head)."""
    lay = layout or ParamLayout.for_model("CNNModel")
    p = params if params.dim() == 2 else params[None]
    return ops.native().cnn2_eval(p.contiguous(), [s.offset for s in lay.slots], rows.contiguous())


class Validation:
    def __init__(self, model_name: str, data_name: str, logger, device="cpu", data_cfg: Optional[dict] = None,
                 dataset=None, verbose: bool = True):
        self.model_name = model_name
        self.data_name = data_name
        self.logger = logger
        self.device = torch.device(device)
        self.verbose = verbose
        self.model = build_model(model_name, seed=0).to(self.device).eval()
        self.layout = ParamLayout.from_state_dict(self.model.state_dict())
        ds = dataset if dataset is not None else resolve_dataset(data_name, "test", data_cfg, verbose=verbose)
        self.table = DeviceTable(ds, self.device)
        self.last_metric: float = float("nan")
        self._runners = {}

    def _program_runner(self, C: int = 1):
        if C not in self._runners:
            from ..fl.programs import ProgramRunner, make_program

            self._runners[C] = ProgramRunner(make_program(self.model_name, C, PROGRAM_EVAL_BATCH[self.model_name],
                                                          self.device, train=False))
        return self._runners[C]

    # -- forward over the whole test set ------------------------------------------------------
    @torch.no_grad()
    def _outputs(self, flat: torch.Tensor) -> torch.Tensor:
        flat = flat.to(self.device, torch.float32)
        if self.data_name == "ICU" and self.model_name == "TransformerModel" and self.device.type == "cuda":
            from ..ops.transformer import eval_forward

            return eval_forward(flat, self.table.rows)
        if self.data_name == "ICU" and self.model_name == "RNNModel" and self.device.type == "cuda":
            from ..ops.rnn import eval_many

            return eval_many(flat[None], self.table.rows)[0]
        if self.data_name == "ICU" and self.model_name == "CNNModel" and self.device.type == "cuda":
            return cnn_eval_many(flat[None], self.table.rows, self.layout)[0]
        if self.device.type == "cuda" and self.model_name in PROGRAM_EVAL_BATCH and self.data_name != "CIFAR10":
            # the layer programs take ICU rows / HAR sequences; images go through the eager model below
            data = self.table.rows if self.data_name == "ICU" else self.table.x
            return self._program_runner().predict(flat[None], data)[0]
        sd = self.layout.unflatten(flat, clone=False)
        self.model.load_state_dict(sd, strict=True)
        outs = []
        chunk = EVAL_CHUNK if self.data_name != "CIFAR10" else 1024
        for a in range(0, self.table.n, chunk):
            idx = torch.arange(a, min(a + chunk, self.table.n), device=self.device)
            if self.data_name == "CIFAR10":
                x, _ = self.table.image_batch(idx)
                outs.append(self.model(x))
            elif self.data_name == "ICU":
                v, l, _ = self.table.icu_batch(idx)
                outs.append(self.model(v, l).reshape(-1))
            else:
                x, _ = self.table.har_batch(idx)
                outs.append(self.model(x))
        return torch.cat(outs, dim=0)

    def _labels(self) -> torch.Tensor:
        return self.table.rows[:, -1] if self.data_name == "ICU" else self.table.y

    def _finish_icu(self, outputs: torch.Tensor, labels: torch.Tensor) -> Tuple[bool, float]:
        auc, has_nan = ops.roc_auc_checked(outputs, labels)
        return self._icu_result(auc, has_nan)

    def _icu_result(self, auc: float, has_nan: bool) -> Tuple[bool, float]:
        if has_nan:
            print_with_color("NaN detected in output, training false", "yellow")
            self.last_metric = float("nan")
            return False, float("nan")
        if self.verbose:
            print(f"ROC_AUC: {auc:.4f}")
        self.logger.log_info(f"ROC_AUC: {auc:.4f}")
        self.last_metric = auc
        return True, auc

    def _finish_image(self, loss_sum: float, correct: int) -> Tuple[bool, float]:
        n = self.table.n
        loss = loss_sum / n
        acc = 100.0 * correct / n
        msg = f"Test set: Average loss: {loss:.4f}, Accuracy: {correct}/{n} ({acc:.2f}%)\n"
        if self.verbose:
            print(msg)
        self.logger.log_info(msg)
        self.last_metric = acc
        if math.isnan(loss) or abs(loss) > 10e5:
            return False, acc
        return True, acc

    def _image_stats(self, flat: torch.Tensor) -> Tuple[float, int]:
        out = self._outputs(flat)
        y = self._labels()
        loss = float(torch.nn.functional.nll_loss(out.float(), y, reduction="sum"))
        return loss, int((out.argmax(dim=1) == y).sum())

    def prefetch(self, flat: torch.Tensor) -> bool:
        """Enqueue the device half of ``test(flat)`` (ICU on a GPU: forward + device ROC-AUC, result copied to pinned
        host memory) on the current stream now; a later ``test`` of the same, unmodified tensor only reads it.
        The engine calls this ahead of a speculative launch whose trainer occupies every CU (cnn2: 32 workgroups
        per client): a validation queued behind that launch on a side stream could not start before it ended,
        and the host, waiting for the metric, then enqueued the round after it late (GPU idle in between)."""
        self._pre = None
        if not (self.device.type == "cuda" and self.data_name == "ICU"):
            return False
        out = self._outputs(flat)
        r = ops.native().roc_auc_dev(out.reshape(-1).float().contiguous(), self._labels().reshape(-1).float().contiguous())
        buf = torch.empty(r.shape, dtype=r.dtype, pin_memory=True)
        buf.copy_(r, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._pre = (flat, flat._version, buf, ev)
        return True

    def test(self, flat: torch.Tensor) -> Tuple[bool, float]:
        pre, self._pre = getattr(self, "_pre", None), None
        if pre is not None and pre[0] is flat and pre[1] == flat._version:
            pre[3].synchronize()
            auc, nan = pre[2].tolist()
            return self._icu_result(auc, nan > 0.5)
        if self.data_name == "CIFAR10":
            return self._finish_image(*self._image_stats(flat))
        out = self._outputs(flat)
        if self.data_name == "ICU":
            return self._finish_icu(out, self._labels())
        pred = out.argmax(dim=1)
        acc = float((pred == self._labels()).float().mean().item())
        if self.verbose:
            print(f"Test Accuracy: {acc:.4f}")
        self.logger.log_info(f"Test Accuracy: {acc:.4f}")
        self.last_metric = acc
        return True, acc

    def test_hyper(self, hnet, num_client: int) -> Tuple[bool, float]:
        if self.data_name == "CIFAR10":
            loss, correct = 0.0, 0
            for i in range(num_client):
                l, c = self._image_stats(hnet.generate(i))
                loss, correct = loss + l, correct + c
            return self._finish_image(loss, correct)
        if self.data_name != "ICU":
            raise ValueError(f"Not found test function for data name {self.data_name}")
        if self.device.type == "cuda" and self.model_name == "RNNModel" and num_client > 0:
            # every client's generated model in ONE fused launch (rnn2.hip k_rnn2_eval)
            from ..ops.rnn import eval_many

            flats = hnet.generate_many(range(num_client)).to(self.device, torch.float32).contiguous()
            out = eval_many(flats, self.table.rows).reshape(-1)
            return self._finish_icu(out, self._labels().repeat(num_client))
        if self.device.type == "cuda" and self.model_name == "CNNModel" and num_client > 0:
            # every client's generated model in ONE fused launch (cnn2.hip k_cnn2_eval)
            flats = hnet.generate_many(range(num_client)).to(self.device, torch.float32).contiguous()
            out = cnn_eval_many(flats, self.table.rows, self.layout).reshape(-1)
            return self._finish_icu(out, self._labels().repeat(num_client))
        if self.device.type == "cuda" and self.model_name in PROGRAM_EVAL_BATCH and num_client > 0:
            # every client's generated model through ONE client-batched eval program
            flats = hnet.generate_many(range(num_client)).to(self.device, torch.float32).contiguous()
            data = self.table.rows
            out = self._program_runner(num_client).predict(flats, data).reshape(-1)
            return self._finish_icu(out, self._labels().repeat(num_client))
        if self.device.type == "cuda" and num_client > 0:
            flats = hnet.generate_many(range(num_client)).to(self.device, torch.float32)  # one GEMM
            if self.model_name == "TransformerModel":
                out = ops.native().tf_eval_many(flats.contiguous(), self.table.rows).reshape(-1)
            else:
                out = torch.cat([self._outputs(flats[i]).reshape(-1) for i in range(num_client)])
            return self._finish_icu(out, self._labels().repeat(num_client))
        outs, labs = [], []
        for i in range(num_client):
            flat = hnet.generate(i)
            outs.append(self._outputs(flat).reshape(-1))
            labs.append(self._labels())
        return self._finish_icu(torch.cat(outs), torch.cat(labs))
