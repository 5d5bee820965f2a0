"""PointSea (models_PointSea/PointSea.py, IJCV'25) restated as a caller of
this package's hot path: the ShapeNet-55 train step of BASELINE.json
configs[4] (partial 2048 -> coarse 256 -> 2048 -> 8192 at step 2/4, merge /
local points 1024) with the PCViews_Real depth renderer
(models_PointSea/mv_utils_zs.py) on libpcops.so.

Module / attribute names follow the reference (encoder.img_feature_extractor
.layer1 ..., refine1.fusionMlp ...), so a reference state_dict loads with
strict=True.  Differences from the reference that do not change values:
  * the ResNet-18 image encoder (PointSea.py:37-61) is built locally with
    torchvision's layout and initialisation (torchvision is absent and its
    ImageNet weights are a remote fetch -- random init, as SURVEY 8c says);
  * the refinement stages run token-major (B, N, C): every 1x1 Conv1d is a
    GEMM on contiguous rows and the reference's raw reshapes are reproduced
    as the equivalent index maps (see SDG.forward_tokens).

Reference map:
  FeatureExtractor (no PCSA)            PointSea.py:11-35
  ResEncoder                            PointSea.py:37-61
  SDG / SDG_l (path selection)          PointSea.py:63-186
  SVFNet (two view attentions)          PointSea.py:188-229
  local_encoder (3 EdgeConvs)           PointSea.py:231-248
  Model                                 PointSea.py:250-272
  SDG_Decoder / self_attention_woinp    models_PointSea/model_utils.py:463-509
"""
import os

import torch
import torch.nn.functional as F
from torch import nn

from .attention import (PosEmbedding, SDG_Decoder_PointSea, _want_bf16, blend, block_sum, cross_attention,
                        self_attention, to_tokens)
from .chamfer3D import chamfer_3DDist
from ._lib import call, fork, lib, ptr, stream_of
from .batchnorm import ACT_RELU, bn_act
from .pointnet2_utils import furthest_point_sample, gather_operation
from .svdformer import (MLP_CONV, BasicBlock, EdgeConv, FeatureExtractor, SinusoidalPositionalEmbedding, _lin,
                        shared_partial_fps)

_LOCAL_FPS_FORK = os.environ.get("PCOPS_LOCAL_FPS_FORK", "0") == "1"


# PCOPS_PS_CAT16=0: the path-selection concatenation in fp32, cast by autocast (A/B)
_CAT16 = os.environ.get("PCOPS_PS_CAT16", "1") != "0"


# ----------------------------------------------------------------- image encoder
class ResEncoder(nn.Module):
    """PointSea.py:37-61: torchvision resnet18 stem + layer1-4 -> (3B, 512, 7, 7)."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        inplanes = 64
        for i, planes in enumerate((64, 128, 256, 512)):
            stride = 1 if i == 0 else 2
            down = None
            if stride != 1 or inplanes != planes:
                down = nn.Sequential(nn.Conv2d(inplanes, planes, 1, stride=stride, bias=False),
                                     nn.BatchNorm2d(planes))
            setattr(self, f"layer{i + 1}", nn.Sequential(BasicBlock(inplanes, planes, stride, down),
                                                         BasicBlock(planes, planes)))
            inplanes = planes
        # torchvision ResNet.__init__ initialisation (zero_init_residual=False)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def forward(self, input_view):
        x = maxpool3s2(self.maxpool, bn_act(self.conv1(input_view), self.bn1, ACT_RELU))
        return self.layer4(self.layer3(self.layer2(self.layer1(x))))


class _MaxPool3s2(torch.autograd.Function):
    """nn.MaxPool2d(3, 2, 1) on a channels_last activation on libpcops (pcops_maxpool3s2_fwd / _bwd):
    torch's NHWC kernels ran this pool on a 3072-thread grid (104 + 149 us per PointSea step)."""

    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        OH, OW = (H + 1) // 2, (W + 1) // 2
        y = torch.empty((N, C, OH, OW), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        arg = torch.empty((N, OH, OW, C), dtype=torch.uint8, device=x.device)
        with torch.cuda.device(x.device):
            call("maxpool3s2_fwd", lib().pcops_maxpool3s2_fwd, ptr(x), _POOL_DT[x.dtype], N, H, W, C, ptr(y), ptr(arg),
                 stream_of(x))
        ctx.save_for_backward(arg)
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, gy):
        (arg,) = ctx.saved_tensors
        N, C, H, W = ctx.shape
        gy = gy.contiguous(memory_format=torch.channels_last)
        gx = torch.empty((N, C, H, W), dtype=gy.dtype, device=gy.device, memory_format=torch.channels_last)
        with torch.cuda.device(gy.device):
            call("maxpool3s2_bwd", lib().pcops_maxpool3s2_bwd, ptr(gy), ptr(arg), _POOL_DT[gy.dtype], N, H, W, C,
                 ptr(gx), stream_of(gy))
        return gx


_POOL_DT = {torch.float32: 0, torch.bfloat16: 1}
_PCOPS_POOL = os.environ.get("PCOPS_POOL", "1") != "0"   # A/B switch


def maxpool3s2(pool, x):
    """pool(x) for the stem's nn.MaxPool2d(3, 2, 1): _MaxPool3s2 on channels_last CUDA fp32 / bf16."""
    if (_PCOPS_POOL and x.is_cuda and x.dim() == 4 and x.dtype in _POOL_DT and x.shape[1] > 0
            and x.is_contiguous(memory_format=torch.channels_last) and pool.kernel_size in (3, (3, 3))
            and pool.stride in (2, (2, 2)) and pool.padding in (1, (1, 1)) and pool.dilation in (1, (1, 1))
            and not pool.ceil_mode and not pool.return_indices):
        return _MaxPool3s2.apply(x)
    return pool(x)


# ----------------------------------------------------------------- refinement
class SDG(nn.Module):
    """PointSea.py:63-124 (SDG) and, with `with_prev=True`, :126-186 (SDG_l):
    structure analysis + similarity alignment + path selection."""

    def __init__(self, channel=128, ratio=1, hidden_dim=768, with_prev=False):
        super().__init__()
        self.channel, self.hidden, self.ratio, self.with_prev = channel, hidden_dim, ratio, with_prev
        self.conv_1 = nn.Conv1d(256, channel, kernel_size=1)
        self.conv_11 = nn.Conv1d(512, 256, kernel_size=1)
        self.conv_x = nn.Conv1d(3, 64, kernel_size=1)
        self.sa1 = self_attention(channel * 2, hidden_dim, dropout=0.0, nhead=8)
        self.cross1 = cross_attention(hidden_dim, hidden_dim, dropout=0.0, nhead=8)
        self.decoder1 = SDG_Decoder_PointSea(hidden_dim, channel, ratio)
        self.decoder2 = SDG_Decoder_PointSea(hidden_dim, channel, ratio)
        self.relu = nn.GELU()
        self.conv_out = nn.Conv1d(64, 3, kernel_size=1)
        self.conv_delta = nn.Conv1d(channel, channel * 1, kernel_size=1)
        self.conv_ps = nn.Conv1d(hidden_dim, channel * ratio, kernel_size=1)
        self.conv_x1 = nn.Conv1d(64, channel, kernel_size=1)
        self.conv_out1 = nn.Conv1d(channel, 64, kernel_size=1)
        self.mlpp = MLP_CONV(in_channel=832, layer_dims=[hidden_dim])
        self.sigma_d = 0.2
        self.embedding = SinusoidalPositionalEmbedding(hidden_dim)
        self.cd_distance = chamfer_3DDist()
        fusion_in = hidden_dim * 2 + channel * (2 if with_prev else 1)
        self.fusionMlp = MLP_CONV(in_channel=fusion_in, layer_dims=[hidden_dim])

    def forward(self, local_feat, coarse, f_g, partial, F_L_Pre=None):
        """Reference signature: (B,832,Nl), (B,3,N), (B,512,1), (B,3,2048)[, (B,128,N)]
        -> (fine (B,3,N*r), F_L (B,128,N*r)) for SDG, fine only for SDG_l."""
        prev = None if F_L_Pre is None else F_L_Pre.transpose(1, 2).contiguous()
        fine, F_L = self.forward_tokens(to_tokens(local_feat), coarse.transpose(1, 2).contiguous(), f_g,
                                        partial.transpose(1, 2).contiguous(), prev)
        fine = fine.transpose(1, 2).contiguous()
        return fine if self.with_prev else (fine, F_L.transpose(1, 2).contiguous())

    def forward_tokens(self, local_tok, coarse, f_g, partial, F_L_prev=None):
        """local_tok (B,Nl,832), coarse (B,N,3), f_g (B,512,1), partial (B,2048,3),
        F_L_prev (B,N,128) -> (fine (B,N*r,3), F_L (B,N*r,128))."""
        B, N, _ = coarse.shape
        Fx = _lin(self.conv_x1, self.relu(_lin(self.conv_x, coarse)))
        g = _lin(self.conv_1, self.relu(_lin(self.conv_11, f_g.transpose(1, 2))))   # (B, 1, channel)
        Fx = torch.cat([Fx, g.expand(B, N, g.shape[-1]).to(Fx.dtype)], dim=-1)
        # structure analysis (PointSea.py:100-105): half Chamfer to the partial input
        half_cd = self.cd_distance(coarse.float().contiguous(), partial.float().contiguous())[0] / self.sigma_d
        pos = PosEmbedding(half_cd, self.embedding, self.hidden)   # added inside the q / k input
        s, f = self.sa1.forward_tokens(Fx, pos)
        F_Q = s + f
        F_Q_ = self.decoder1.forward_tokens(F_Q)           # PointSea's decoder ignores pos
        f_g_current = F_Q.max(dim=1, keepdim=True)[0]      # torch.max(F_Q, 2)[0]
        # similarity alignment
        local = _lin(self.mlpp.mlp[0], local_tok)
        s, f = self.cross1.forward_tokens(F_Q, local)
        F_H_ = self.decoder2.forward_tokens((s, f))        # its first op is a LayerNorm of s + f
        # path selection
        if _CAT16 and F_Q_.is_cuda and _want_bf16():
            # the concatenation only feeds fusionMlp's GEMM: built from parts already in the bf16
            # operand dtype (cat of bf16 parts == bf16 of the fp32 cat), the sum rounded once in its add
            parts = [block_sum(F_Q_, F_H_)]
            if self.with_prev:
                parts.append(F_L_prev.to(torch.bfloat16))
            parts += [f_g_current.expand(B, N, -1).to(torch.bfloat16), g.expand(B, N, -1).to(torch.bfloat16)]
        else:
            parts = [F_Q_ + F_H_]
            if self.with_prev:
                parts.append(F_L_prev.to(parts[0].dtype))
            parts += [f_g_current.expand(B, N, -1).to(parts[0].dtype), g.expand(B, N, -1).to(parts[0].dtype)]
        score = torch.sigmoid(_lin(self.fusionMlp.mlp[0], torch.cat(parts, dim=-1)))
        F_L = blend(score, F_Q_, F_H_, gemm_only=True)     # score * F_Q_ + (1 - score) * F_H_; read by conv_ps only
        # conv_ps(F_L).reshape(B, C, N*r): point j*N + n takes channels c*r + j of point n
        T = _lin(self.conv_ps, F_L)
        r = self.ratio
        F_L = _lin(self.conv_delta, T.reshape(B, N, -1, r).permute(0, 3, 1, 2).reshape(B, r * N, -1))
        O_L = _lin(self.conv_out, self.relu(_lin(self.conv_out1, F_L)))
        return coarse.repeat(1, r, 1) + O_L, F_L


class SDG_l(SDG):
    """PointSea.py:126-186 (path selection also sees the previous stage's F_L)."""

    def __init__(self, channel=128, ratio=1, hidden_dim=512):
        super().__init__(channel, ratio, hidden_dim, with_prev=True)


# ----------------------------------------------------------------- encoders
class SVFNet(nn.Module):
    """PointSea.py:188-229: ResNet-18 view tokens + point features, two view attentions."""

    def __init__(self, cfg):
        super().__init__()
        self.channel = 64
        self.point_feature_extractor = FeatureExtractor(use_pcsa=False)
        self.view_distance = cfg.NETWORK.view_distance
        self.relu = nn.GELU()
        self.sa = self_attention(self.channel * 8, self.channel * 8, dropout=0.0)
        self.viewattn1 = self_attention(256 + 512, 512)
        self.viewattn2 = self_attention(256 + 512, 256)
        self.conv_out = nn.Conv1d(64, 3, kernel_size=1)
        self.conv_out1 = nn.Conv1d(512 + self.channel * 4, 64, kernel_size=1)
        self.ps = nn.ConvTranspose1d(512, self.channel, 128, bias=True)
        self.ps_refuse = nn.Conv1d(512 + self.channel, self.channel * 8, kernel_size=1)
        self.img_feature_extractor = ResEncoder()
        self.posmlp = MLP_CONV(3, [64, 256])
        d = self.view_distance
        self.register_buffer("view_point", torch.tensor([0, 0, -d, -d, 0, 0, 0, d, 0], dtype=torch.float32)
                             .view(-1, 3, 3).permute(0, 2, 1).contiguous(), persistent=False)

    def forward(self, points, depth, fidx=None):
        B, _, N = points.size()
        f_v = self.img_feature_extractor(depth.contiguous(memory_format=torch.channels_last))
        f_v = f_v.flatten(2)                                           # 'bv c h w -> bv c (h w)'
        f_p = self.point_feature_extractor(points, fidx=fidx)          # (B, 256, 1)
        view_feature_1 = self.posmlp(self.view_point.expand(B, 3, 3))  # (B, 256, 3)
        # f_p.repeat(3, 1, n): image r (= 3b + v) is paired with f_p[r % B], as in the reference
        f_v_ = self.viewattn1(torch.cat([f_v, f_p.repeat(3, 1, f_v.size(2)).to(f_v.dtype)], 1))
        C = f_v_.shape[1]
        f_v_ = f_v_.view(B, 3, C, -1).max(dim=3)[0].transpose(1, 2)   # '(b v) c n -> b c v n', max n
        f_v_ = self.viewattn2(torch.cat([f_v_, f_p.repeat(1, 1, f_v_.size(2)).to(f_v_.dtype)], dim=1),
                              view_feature_1.permute(2, 0, 1))
        f_v_ = F.adaptive_max_pool1d(f_v_, 1)
        f_g = torch.cat([f_p, f_v_.to(f_p.dtype)], 1)
        x = self.relu(self.ps(f_g))
        x = self.relu(self.ps_refuse(torch.cat([x, f_g.repeat(1, 1, x.size(2)).to(x.dtype)], 1)))
        x2_d = (self.sa(x)).reshape(B, self.channel * 4, N // 8)
        coarse = self.conv_out(self.relu(self.conv_out1(torch.cat([x2_d, f_g.repeat(1, 1, x2_d.size(2))
                                                                   .to(x2_d.dtype)], 1))))
        return f_g, coarse


class local_encoder(nn.Module):
    """PointSea.py:231-248 -> (B, 64+256+512, local_points)."""

    def __init__(self, cfg):
        super().__init__()
        self.gcn_1 = EdgeConv(3, 64, 16)
        self.gcn_2 = EdgeConv(64, 256, 8)
        self.gcn_3 = EdgeConv(256, 512, 4)
        self.local_number = cfg.NETWORK.local_points

    def forward(self, inp, fidx=None):
        """fidx: a model_utils.SharedFPS of inp (the model's shared partial-cloud FPS)."""
        if fidx is not None:
            x1 = self.gcn_1(inp)
            x1 = gather_operation(x1.float().contiguous(), fidx.take(self.local_number))
            x2 = self.gcn_2(x1)
            x3 = self.gcn_3(x2)
            return torch.cat([x1, x2.to(x1.dtype), x3.to(x1.dtype)], 1)
        # the FPS depends on the input cloud only: PCOPS_LOCAL_FPS_FORK=1 runs it on a stream of its
        # own (lane 3) beside gcn_1.  This block already runs in the model's lane-0 fork; `inp` was
        # produced before that fork, so the inner fork may start from the outer fork's origin
        # stream -- the form that stays capturable (_lib.fork)
        if _LOCAL_FPS_FORK:
            with fork(inp.device, lane=3, inputs=(inp,), base="outer") as br:
                idx = furthest_point_sample(inp.transpose(1, 2).float().contiguous(), self.local_number)
            x1 = self.gcn_1(inp)
            idx = br.join(idx)
        else:
            x1 = self.gcn_1(inp)
            idx = furthest_point_sample(inp.transpose(1, 2).float().contiguous(), self.local_number)
        x1 = gather_operation(x1.float().contiguous(), idx)
        x2 = self.gcn_2(x1)
        x3 = self.gcn_3(x2)
        return torch.cat([x1, x2.to(x1.dtype), x3.to(x1.dtype)], 1)


class Model(nn.Module):
    """PointSea.py:250-272: (partial (B,N,3), depth (3B,3,224,224)) -> (coarse, fine1, fine2)."""

    def __init__(self, cfg):
        super().__init__()
        self.encoder = SVFNet(cfg)
        self.localencoder = local_encoder(cfg)
        self.merge_points = cfg.NETWORK.merge_points
        self.refine1 = SDG(ratio=cfg.NETWORK.step1)
        self.refine2 = SDG_l(ratio=cfg.NETWORK.step2)
        for m in self.modules():   # NHWC 2-D convs (see svdformer.Model)
            if isinstance(m, nn.Conv2d):
                m.to(memory_format=torch.channels_last)

    def forward(self, partial, depth):
        partial_cm = partial.transpose(1, 2).contiguous()
        # the local encoder (EdgeConv kNN, FPS, 1x1-conv GEMMs on rocBLAS: no stream-K)
        # only depends on the partial cloud: it runs on a second HIP stream
        # beside the view/point encoder
        with fork(partial.device, inputs=(partial_cm, partial)) as br:
            # the partial cloud's FPS once, first on this stream: the local encoder's 1024 and the
            # point encoder's SA module's first 512 (svdformer.shared_partial_fps)
            fidx = shared_partial_fps(partial, self.localencoder.local_number,
                                      self.encoder.point_feature_extractor.sa_module_1.npoint)
            local_feat = self.localencoder(partial_cm, fidx=fidx)
        feat_g, coarse = self.encoder(partial_cm, depth, fidx=fidx)
        local_feat = br.join(local_feat)
        coarse_merge = torch.cat([partial_cm, coarse.to(partial_cm.dtype)], dim=2).float().contiguous()
        coarse_merge = gather_operation(coarse_merge, furthest_point_sample(coarse_merge.transpose(1, 2).contiguous(),
                                                                            self.merge_points))
        local_tok = to_tokens(local_feat)
        partial = partial.contiguous()
        fine1, F_L_1 = self.refine1.forward_tokens(local_tok, coarse_merge.transpose(1, 2).contiguous(), feat_g,
                                                   partial)
        fine2, _ = self.refine2.forward_tokens(local_tok, fine1, feat_g, partial, F_L_1)
        return coarse.transpose(1, 2).contiguous(), fine1, fine2


class Config55:
    """The NETWORK keys of config_55.py:53-59 the model reads (TRAIN.BATCH_SIZE :65 = 16)."""

    class NETWORK:
        step1 = 2
        step2 = 4
        merge_points = 1024
        local_points = 1024
        view_distance = 1.5
        USE_PCSA = True

    class TRAIN:
        BATCH_SIZE = 16
