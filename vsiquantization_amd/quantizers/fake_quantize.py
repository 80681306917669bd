"""FakeQuantize layer base (reference: quantizers/fake_quantize.py:8-66).

Holds ``weight_quantizer`` and ``activation_quantizer`` (QuantizationManagers,
learnable by default as in the reference, fake_quantize.py:22-36) and runs
``[quantize input] -> quantize weight -> run_forward_core -> [quantize output]``.
Subclasses (modules/fused.py) provide ``run_forward_core`` and the wrapped
conv/linear as ``conv_fuse`` / ``linear_fuse``.
"""
import torch.nn as nn

from .quantization_manager import QuantizationManager


class FakeQuantize(nn.Module):
    def __init__(self, observer_w_name: str, quantizer_w_name: str, observer_a_name: str,
                 quantizer_a_name: str, w_symmetric: bool = True, a_symmetric: bool = True,
                 bits_w: int = 4, bits_a: int = 8, quantize_out: bool = True,
                 quantize_inp: bool = False):
        super().__init__()
        self.weight_quantizer = QuantizationManager(quantizer_w_name, observer_w_name, bits_w,
                                                    w_symmetric, is_learning_scale=True)
        self.activation_quantizer = QuantizationManager(quantizer_a_name, observer_a_name, bits_a,
                                                        a_symmetric, is_learning_scale=True)
        self.bits_w = bits_w
        self.bits_a = bits_a
        self.quantize_out = quantize_out
        self.quantize_inp = quantize_inp

    def forward(self, x):
        if self.quantize_inp:
            x = self.quantize_activation(x)
        w, b = self.get_weight_bias()
        out = self.run_forward_core(x, self.quantize_weights(w), b)
        if self.quantize_out:
            out = self.quantize_activation(out)
        return out

    def run_forward_core(self, x, weights, bias):
        raise NotImplementedError

    def get_weight_bias(self):
        conv = self.conv_fuse
        return conv.weight, conv.bias

    def quantize_weights(self, weights):
        # a result precomputed by a multi-tensor launch (quantizers/foreach.py) for exactly
        # this weight tensor is used once; anything else takes the per-layer path
        stash = self.__dict__.pop("_weight_stash", None)
        if stash is not None and stash[0] is weights:
            return stash[1]
        return self.weight_quantizer.quantize(weights)

    def quantize_activation(self, out):
        return self.activation_quantizer.quantize(out)
