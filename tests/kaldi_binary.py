"""An independent encoder of Kaldi's binary stream format (upstream
base/io-funcs.h / io-funcs-inl.h, matrix/kaldi-matrix.cc, kaldi-vector.cc),
written from the format's definition -- not from kaldi-lite -- and the
components' token sequences as the reference writes them
(nnet0/nnet-component-nnet0.cc:620-666 Conv, :936-959 Maxpool, :1001-1020 FC;
nnet2/nnet-component.cc:398-412 NonlinearComponent, :2854-2866 Splice).

  token        "<Tok>" + " "
  int32        size byte 4, 4 bytes little-endian
  float        size byte 4, IEEE single;  double: size byte 8, IEEE double
  bool         "T" / "F" (no separator in binary mode)
  matrix       token "FM", int32 rows, int32 cols, rows x cols floats
  vector       token "FV" (floats) / "DV" (doubles), int32 dim, the values
  int vector   size byte 4, raw int32 count, raw int32 values
  file header  "\\0B"
"""
import struct

import numpy as np


def token(t):
    return t.encode() + b" "


def i32(v):
    return b"\x04" + struct.pack("<i", v)


def f32(v):
    return b"\x04" + struct.pack("<f", v)


def f64(v):
    return b"\x08" + struct.pack("<d", v)


def boolean(v):
    return b"T" if v else b"F"


def fmat(a):
    a = np.ascontiguousarray(a, np.float32)
    return token("FM") + i32(a.shape[0]) + i32(a.shape[1]) + a.tobytes()


def fvec(v):
    v = np.ascontiguousarray(v, np.float32)
    return token("FV") + i32(v.size) + v.tobytes()


def dvec(v):
    v = np.ascontiguousarray(v, np.float64)
    return token("DV") + i32(v.size) + v.tobytes()


def ivec(v):
    return b"\x04" + struct.pack("<i", len(v)) + struct.pack(f"<{len(v)}i", *v)


HEADER = b"\x00B"


def conv(p):
    out = token("<ConvolutionComponent>")
    for tok, key in (("<in_height>", "H"), ("<in_width>", "W"), ("<in_channel>", "C"),
                     ("<kernel_height>", "kh"), ("<kernel_width>", "kw"), ("<stride>", "stride"),
                     ("<padding_height>", "ph"), ("<padding_width>", "pw"), ("<group>", "G"),
                     ("<out_height>", "oh"), ("<out_width>", "ow")):
        out += token(tok) + i32(int(p[key]))
    out += token("<LearningRate>") + f32(float(p["lr"]))
    out += token("<WeightDecay>") + f32(float(p["wd"]))
    out += token("<Momentum>") + f32(float(p["m"]))
    out += token("<LinearParams>") + fmat(p["linear"])
    out += token("<BiasParams>") + fvec(p["b"])
    out += token("<PrevGrad>") + fmat(p["prev"])
    out += token("<IsGradient>") + boolean(False)
    return out + token("</ConvolutionComponent>")


def maxpool(p):
    out = token("<MaxpoolComponent>")
    for tok, key in (("<InputDim>", "input_dim"), ("<in_height>", "H"), ("<in_width>", "W"),
                     ("<in_channel>", "C"), ("<OutputDim>", "output_dim"),
                     ("<PoolHeightDim>", "ph"), ("<PoolWidthDim>", "pw"),
                     ("<PoolChannelDim>", "pc")):
        out += token(tok) + i32(int(p[key]))
    out += token("<Overlap>") + boolean(bool(p["overlap"]))
    out += token("<Overlap2D>") + boolean(bool(p["overlap2D"]))
    return out + token("</MaxpoolComponent>")


def fc(p):
    out = token("<FullyConnectedComponent>")
    out += token("<LearningRate>") + f32(float(p["lr"]))
    out += token("<LinearParams>") + fmat(p["linear"])
    out += token("<BiasParams>") + fvec(p["b"])
    out += token("<WeightDecay>") + f32(float(p["wd"]))
    out += token("<Momentum>") + f32(float(p["m"]))
    out += token("<PrevGrad>") + fmat(p["prev"])
    return out + token("</FullyConnectedComponent>")


def relu(p):
    out = token("<RectifiedLinearComponent>") + token("<Dim>") + i32(int(p["dim"]))
    out += token("<ValueSum>") + dvec(p["value_sum"])
    out += token("<DerivSum>") + dvec(p["deriv_sum"])
    out += token("<Count>") + f64(float(p["count"]))
    return out + token("</RectifiedLinearComponent>")


def splice(p):
    out = token("<SpliceComponent>") + token("<InputDim>") + i32(int(p["input_dim"]))
    out += token("<Context>") + ivec([int(c) for c in p["context"]])
    out += token("<ConstComponentDim>") + i32(int(p["const_dim"]))
    return out + token("</SpliceComponent>")


ENCODERS = {"conv": conv, "maxpool": maxpool, "fc": fc, "relu": relu, "splice": splice}


def encode(kind, params):
    return HEADER + ENCODERS[kind](params)
