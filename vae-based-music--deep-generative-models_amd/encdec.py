"""Encoder / decoder stacks — drop-in for the reference encdec.py.

encdec.py:17-41   EncoderConvBlock: down_depth x [Conv1D(embed_width, 2*stride, strides=stride) ->
                  DilatedResnet1D], then Conv1D(output_dim, 3)
encdec.py:44-71   DecoderConvBlock: Conv1D(embed_width, 3), then down_depth x [reversed DilatedResnet1D ->
                  Conv1DTranspose(embed_width or output_dim on the last step, 2*stride, strides=stride)]
encdec.py:74-108  Encoder: `depth` EncoderConvBlocks in order
encdec.py:114-151 Decoder: the blocks in reverse order, then Conv1D(output_dim, 3) to audio channels
Every conv is a libvqa HIP kernel; the audio-side tensors (1 channel) stay fp32.
"""
from __future__ import annotations

import torch

import vqa_lib as V
from resnet import DilatedResnet1D
from vqa_layers import Conv1D, Conv1DTranspose
from vqa_module import Layer


def print_dec_layer(decoder):
    """encdec.py:7-14 debug print of the decoder's dilated layers."""
    for blk in decoder.blocks:
        print(f"-----{blk.prefix}-----")
        for res in blk.res:
            for rb in res.blocks:
                print(f"---------{rb.conv_a.name} (dilation {rb.dilation})---------")


class EncoderConvBlock(Layer):
    def __init__(self, output_dim, embed_width, embed_depth, dilation_factor=1, stride=2, down_depth=4, **kwargs):
        super().__init__(**kwargs)
        self.output_dim, self.embed_width, self.stride, self.down_depth = output_dim, embed_width, stride, down_depth
        self.kernel_size = stride * 2
        self.res = [DilatedResnet1D(embed_width, embed_depth, dilation_factor=dilation_factor) for _ in range(down_depth)]
        self._saved = None

    def _build(self, store, prefix, input_dim):
        self.prefix = prefix
        self.down = []
        cin = input_dim
        for i in range(self.down_depth):
            self.down.append(Conv1D(store, f"{prefix}/down{i}", cin, self.embed_width, self.kernel_size, self.stride))
            self.res[i].build(store, f"{prefix}/res{i}", self.embed_width, self.cdt)
            cin = self.embed_width
        self.proj = Conv1D(store, f"{prefix}/proj", self.embed_width, self.output_dim, 3)
        return self.output_dim

    def forward(self, x, save=False):
        ins = []
        for down, res in zip(self.down, self.res):
            ins.append(x)
            x = res.forward(down.forward(x, self.cdt), save)
        ins.append(x)
        self._saved = ins if save else None
        return self.proj.forward(x, self.cdt)

    def backward(self, dy, need_dx=True):
        ins = self._saved
        self._saved = None
        self.proj.backward_weight(ins[-1], dy, self.cdt)
        g = self.proj.backward_data(dy, ins[-1].shape[1], self.cdt)
        for i in reversed(range(self.down_depth)):
            g = self.res[i].backward(g)
            self.down[i].backward_weight(ins[i], g, self.cdt)
            if i > 0 or need_dx:
                g = self.down[i].backward_data(g, ins[i].shape[1], self.cdt, out_dtype=ins[i].dtype)
            else:
                g = None
        return g


class DecoderConvBlock(Layer):
    def __init__(self, output_dim, embed_width, embed_depth, dilation_factor=1, reverse_dilation=True,
                 dilation_cycle=None, stride=2, down_depth=4, **kwargs):
        super().__init__(**kwargs)
        self.output_dim, self.embed_width, self.stride, self.down_depth = output_dim, embed_width, stride, down_depth
        self.kernel_size = stride * 2
        self.res = [DilatedResnet1D(embed_width, embed_depth, dilation_factor=dilation_factor,
                                    reverse_dilation=reverse_dilation, dilation_cycle=dilation_cycle)
                    for _ in range(down_depth)]
        self._saved = None

    def _build(self, store, prefix, input_dim):
        self.prefix = prefix
        self.pre = Conv1D(store, f"{prefix}/pre", input_dim, self.embed_width, 3)
        self.up = []
        for i in range(self.down_depth):
            self.res[i].build(store, f"{prefix}/res{i}", self.embed_width, self.cdt)
            cout = self.output_dim if i == self.down_depth - 1 else self.embed_width
            self.up.append(Conv1DTranspose(store, f"{prefix}/up{i}", self.embed_width, cout, self.kernel_size,
                                           self.stride))
        return self.output_dim

    def forward(self, x, save=False, stop_before_last_up=False):
        """stop_before_last_up: return the input of the last up conv (the Decoder runs that conv fused with
        its output conv, vqa_dtail)."""
        ins = [x]
        x = self.pre.forward(x, self.cdt)
        for i, (res, up) in enumerate(zip(self.res, self.up)):
            x = res.forward(x, save)
            ins.append(x)
            if stop_before_last_up and i == self.down_depth - 1:
                break
            x = up.forward(x, self.cdt)
        self._saved = ins if save else None
        return x

    def backward(self, dy, skip_last_up=False):
        """skip_last_up: dy is already the gradient of the last up conv's input (fused decoder tail)."""
        ins = self._saved
        self._saved = None
        for i in reversed(range(self.down_depth)):
            if not (skip_last_up and i == self.down_depth - 1):
                self.up[i].backward_weight(ins[i + 1], dy, self.cdt)
                dy = self.up[i].backward_data(dy, self.cdt)
            dy = self.res[i].backward(dy)
        self.pre.backward_weight(ins[0], dy, self.cdt)
        return self.pre.backward_data(dy, ins[0].shape[1], self.cdt)


class Encoder(Layer):
    def __init__(self, output_dim, residual_width, residual_depth, depth, down_depth, strides, dilation_factor=1,
                 **kwargs):
        super().__init__(**kwargs)
        assert depth == len(down_depth), f"Depth {depth} not Legit"  # encdec.py:84-85
        assert depth == len(strides), f"Depth {depth} not Legit"
        self.depth, self.down_depth, self.strides = depth, list(down_depth), list(strides)
        self.blocks = [EncoderConvBlock(output_dim, residual_width, residual_depth, stride=s,
                                        dilation_factor=dilation_factor, down_depth=d)
                       for d, s in zip(down_depth, strides)]

    def _build(self, store, prefix, input_dim):
        dim = input_dim
        for b, blk in enumerate(self.blocks):
            dim = blk.build(store, f"{prefix}/blk{b}", dim, self.cdt)
        return dim

    def forward(self, x, save=False):
        for blk in self.blocks:
            x = blk.forward(x, save)
        return x

    def backward(self, dy, need_dx=False):
        for b in reversed(range(self.depth)):
            dy = self.blocks[b].backward(dy, need_dx=(b > 0 or need_dx))
        return dy


class Decoder(Layer):
    def __init__(self, output_dim, embed_width, residual_width, residual_depth, depth, down_depth, strides,
                 dilation_factor=1, reverse_dilation=True, **kwargs):
        super().__init__(**kwargs)
        assert depth == len(down_depth), f"Depth {depth} not Legit"  # encdec.py:84-85 (Decoder :122-123)
        assert depth == len(strides), f"Depth {depth} not Legit"
        self.depth, self.output_dim, self.embed_width = depth, output_dim, embed_width
        # encdec.py:142: blocks in reverse order of the encoder's (block index b kept for naming)
        self.order = list(reversed(range(depth)))
        self.blocks = [DecoderConvBlock(embed_width, residual_width, residual_depth, stride=strides[b],
                                        dilation_factor=dilation_factor, reverse_dilation=reverse_dilation,
                                        down_depth=down_depth[b]) for b in self.order]
        self._saved = None

    def _build(self, store, prefix, input_dim):
        dim = input_dim
        for b, blk in zip(self.order, self.blocks):
            dim = blk.build(store, f"{prefix}/blk{b}", dim, self.cdt)
        self.out = Conv1D(store, f"{prefix}/out", dim, self.output_dim, 3)
        return self.output_dim

    # run the last up conv and the output conv as one composed thin conv (vqa_dtail.hip) when they fit it
    fuse_tail = True

    def _tail(self):
        up = self.blocks[-1].up[-1]
        out = self.out
        ok = (self.fuse_tail and out.cin == up.cout and out.s == 1 and out.d == 1 and
              V.dtail_supported(up.cin, up.cout, up.K, up.s, out.K, out.cout, V.dtype_code(self.cdt)))
        return (up, out) if ok else None

    def forward(self, x, save=False):
        tail = self._tail()
        last = len(self.blocks) - 1
        for i, blk in enumerate(self.blocks):
            x = blk.forward(x, save, stop_before_last_up=tail is not None and i == last)
        if tail is not None:
            up, out = tail
            B, T, _ = x.shape
            y = torch.empty((B, 2 * T, 1), dtype=torch.float32, device=x.device)
            V.dtail_fwd(x, up.w, up.b, out.w, out.b, y)  # encdec.py:67-68 + :148 composed
            self._saved = ("tail", x) if save else None
            return y
        self._saved = x if save else None
        return self.out.forward(x, self.cdt, out_dtype=torch.float32)

    def backward(self, dy):
        saved = self._saved
        self._saved = None
        if isinstance(saved, tuple):
            h = saved[1]
            up, out = self._tail()
            g = torch.empty_like(h)
            st = self.store
            V.dtail_bwd(dy.contiguous(), h, up.w, up.b, out.w, out.b, g, st.grad_view(f"{up.name}/kernel"),
                        st.grad_view(f"{up.name}/bias"), st.grad_view(f"{out.name}/kernel"),
                        st.grad_view(f"{out.name}/bias"))
            last = len(self.blocks) - 1
            for i in reversed(range(len(self.blocks))):
                g = self.blocks[i].backward(g, skip_last_up=(i == last))
            return g
        g = self.out.backward_data_weight(dy, saved, self.cdt)  # one pass: dx and dW/db (vqa_conv_ends.hip)
        for blk in reversed(self.blocks):
            g = blk.backward(g)
        return g
