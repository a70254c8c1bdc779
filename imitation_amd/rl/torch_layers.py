"""Feature extractors and MLP trunks (SB3 ``torch_layers`` surface).

* :class:`FlattenExtractor`, :class:`CombinedExtractor` (Dict obs), :class:`NatureCNN`
  (the DAgger-Pong config);
* :class:`MlpExtractor` -- separate policy/value trunks with SB3's state-dict
  key layout (``mlp_extractor.{policy,value}_net.{0,2}.*``) so
  ``policy.pth`` files from SB3 ``model.zip`` archives load by name.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Tuple, Type, Union

import torch as th
from torch import nn

from imitation_amd.envs import spaces
from imitation_amd.rl.preprocessing import get_flattened_obs_dim, is_image_space, is_image_space_channels_first


class BaseFeaturesExtractor(nn.Module):
    def __init__(self, observation_space: spaces.Space, features_dim: int = 0):
        super().__init__()
        assert features_dim > 0
        self._observation_space = observation_space
        self._features_dim = features_dim

    @property
    def features_dim(self) -> int:
        return self._features_dim


class FlattenExtractor(BaseFeaturesExtractor):
    def __init__(self, observation_space: spaces.Space):
        super().__init__(observation_space, get_flattened_obs_dim(observation_space))
        self.flatten = nn.Flatten()

    def forward(self, observations: th.Tensor) -> th.Tensor:
        return self.flatten(observations)


class NatureCNN(BaseFeaturesExtractor):
    """Mnih et al. 2015 conv trunk: 8x8s4 -> 4x4s2 -> 3x3s1 -> Linear(512)."""

    def __init__(self, observation_space: spaces.Space, features_dim: int = 512, normalized_image: bool = False):
        super().__init__(observation_space, features_dim)
        # Channel-last frames (the native Atari env's (84, 84, 4)) are consumed as they are:
        # permuting NHWC to logical NCHW is a view whose memory *is* channels_last, so no
        # VecTransposeImage copy is needed in front of the policy.
        self.channels_last_input = not is_image_space_channels_first(observation_space)
        shape = tuple(observation_space.shape)
        n_input_channels = shape[-1] if self.channels_last_input else shape[0]
        chw = (shape[2], shape[0], shape[1]) if self.channels_last_input else shape
        self.cnn = nn.Sequential(
            nn.Conv2d(n_input_channels, 32, kernel_size=8, stride=4, padding=0),
            nn.ReLU(),
            nn.Conv2d(32, 64, kernel_size=4, stride=2, padding=0),
            nn.ReLU(),
            nn.Conv2d(64, 64, kernel_size=3, stride=1, padding=0),
            nn.ReLU(),
            nn.Flatten(),
        )
        with th.no_grad():
            n_flatten = self.cnn(th.zeros((1,) + chw)).shape[1]
        self.linear = nn.Sequential(nn.Linear(n_flatten, features_dim), nn.ReLU())

    def forward(self, observations: th.Tensor, in_scale: float = 1.0) -> th.Tensor:
        # conv trunk: NHWC implicit-GEMM MFMA kernels on GPU (ops/conv.py, csrc/kernels/conv.hip),
        # fp32 reference on CPU; the module keeps SB3's state-dict layout (cnn.{0,2,4}, linear.0).
        # ``in_scale``: raw uint8 frames with the image normalisation (1/255) folded into the
        # first layer's operand load (see BaseModel.extract_features)
        from imitation_amd.ops import conv as conv_ops

        x = observations if self.channels_last_input else observations.permute(0, 2, 3, 1)
        convs = [m for m in self.cnn if isinstance(m, nn.Conv2d)]
        lin = self.linear[0]
        if (x.is_cuda and isinstance(self.linear[-1], nn.ReLU) and len(self.linear) == 2
                and conv_ops.fc_supported(tuple(x.shape), [c.weight for c in convs], [c.stride[0] for c in convs],
                                          lin.out_features)):
            # whole extractor (convs + flatten + Linear + ReLU) as one kernel-backed node
            return conv_ops.conv_stack_fc(x, [c.weight for c in convs], [c.bias for c in convs],
                                          [c.stride[0] for c in convs], lin.weight, lin.bias, in_scale)
        y = conv_ops.conv_stack(x, [c.weight for c in convs], [c.bias for c in convs], [c.stride[0] for c in convs],
                                in_scale)
        y = y.permute(0, 3, 1, 2).reshape(y.shape[0], -1)  # nn.Flatten order (C, H, W)
        return self.linear(y)

    def raw_frames_ok(self, obs) -> bool:
        """Whether ``obs`` (un-preprocessed) can go to :meth:`forward` as uint8 with in_scale
        1/255: channel-last frames on the GPU kernel path."""
        from imitation_amd.ops import conv as conv_ops
        from imitation_amd import ops

        if not (isinstance(obs, th.Tensor) and obs.dtype == th.uint8 and obs.is_cuda and obs.dim() == 4
                and self.channels_last_input and ops.use_kernel(obs)):
            return False
        convs = [m for m in self.cnn if isinstance(m, nn.Conv2d)]
        return conv_ops.supported(tuple(obs.shape), [c.weight for c in convs], [c.stride[0] for c in convs])


class CombinedExtractor(BaseFeaturesExtractor):
    """Dict observations: NatureCNN per image key, flatten otherwise, concatenated."""

    def __init__(self, observation_space: spaces.Dict, cnn_output_dim: int = 256, normalized_image: bool = False):
        super().__init__(observation_space, features_dim=1)
        extractors: Dict[str, nn.Module] = {}
        total = 0
        for key, sub in observation_space.spaces.items():
            if is_image_space(sub, normalized_image=normalized_image):
                extractors[key] = NatureCNN(sub, features_dim=cnn_output_dim, normalized_image=normalized_image)
                total += cnn_output_dim
            else:
                extractors[key] = nn.Flatten()
                total += get_flattened_obs_dim(sub)
        self.extractors = nn.ModuleDict(extractors)
        self._features_dim = total

    def forward(self, observations: Dict[str, th.Tensor]) -> th.Tensor:
        return th.cat([ext(observations[k]) for k, ext in self.extractors.items()], dim=1)


def create_mlp(
    input_dim: int,
    output_dim: int,
    net_arch: List[int],
    activation_fn: Type[nn.Module] = nn.ReLU,
    squash_output: bool = False,
    with_bias: bool = True,
) -> List[nn.Module]:
    modules: List[nn.Module] = []
    last = input_dim
    for h in net_arch:
        modules += [nn.Linear(last, h, bias=with_bias), activation_fn()]
        last = h
    if output_dim > 0:
        modules.append(nn.Linear(last, output_dim, bias=with_bias))
    if squash_output:
        modules.append(nn.Tanh())
    return modules


class MlpExtractor(nn.Module):
    """Separate policy / value trunks (``net_arch`` list -> both, dict -> ``pi``/``vf``)."""

    def __init__(
        self,
        feature_dim: int,
        net_arch: Union[List[int], Dict[str, List[int]]],
        activation_fn: Type[nn.Module],
        device: Union[th.device, str] = "auto",
    ):
        super().__init__()
        if isinstance(net_arch, dict):
            pi_dims, vf_dims = net_arch.get("pi", []), net_arch.get("vf", [])
        else:
            pi_dims = vf_dims = list(net_arch)
        self.activation_fn = activation_fn
        pol: List[nn.Module] = []
        val: List[nn.Module] = []
        last_pi = last_vf = feature_dim
        for d in pi_dims:
            pol += [nn.Linear(last_pi, d), activation_fn()]
            last_pi = d
        for d in vf_dims:
            val += [nn.Linear(last_vf, d), activation_fn()]
            last_vf = d
        self.latent_dim_pi = last_pi
        self.latent_dim_vf = last_vf
        self.policy_net = nn.Sequential(*pol)
        self.value_net = nn.Sequential(*val)

    def forward(self, features: th.Tensor) -> Tuple[th.Tensor, th.Tensor]:
        return self.forward_actor(features), self.forward_critic(features)

    def forward_actor(self, features: th.Tensor) -> th.Tensor:
        return self.policy_net(features)

    def forward_critic(self, features: th.Tensor) -> th.Tensor:
        return self.value_net(features)


def get_actor_critic_arch(net_arch: Union[List[int], Dict[str, List[int]]]) -> Tuple[List[int], List[int]]:
    if isinstance(net_arch, list):
        return list(net_arch), list(net_arch)
    assert isinstance(net_arch, dict)
    return list(net_arch["pi"]), list(net_arch["qf"])
