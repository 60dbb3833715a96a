"""Policy in the loop (BASELINE config 5): the ttrl_agent DQN ego-attention network,
batched over every env of the simulator and fed the Kinematics observation in place.

Restates ttrl_agent/agents/common/models.py — MultiLayerPerceptron (:50-76),
EgoAttention (:157-194), EgoAttentionNetwork (:237-312), attention (:370-388) — and the
acting side of the DQN agent: AbstractDQNAgent.act (deep_q_network/abstract.py:65-83)
with EpsilonGreedy exploration (exploration/epsilon_greedy.py:7-57; schedule from
scripts/configs/IntersectionEnv/agents/DQNAgent/baseline.json:12-17).  The forward is a
dense contraction (7->64->64 embeddings, 2-head attention over 15 entities, 64->64->64->n
head): it runs as torch GEMMs on the same HIP stream as the simulator (hipBLASLt/MFMA),
no host round trip between env.step and the next action.
"""
from __future__ import annotations

import math

import torch
from torch import nn
from torch.nn import functional as F

EGO_ATTENTION_2H = {  # configs/IntersectionEnv/agents/DQNAgent/ego_attention.json + ego_attention_2h.json
    "type": "EgoAttentionNetwork",
    "presence_feature_idx": 0,
    "embedding_layer": {"type": "MultiLayerPerceptron", "layers": [64, 64], "reshape": False, "in": 7},
    "others_embedding_layer": {"type": "MultiLayerPerceptron", "layers": [64, 64], "reshape": False, "in": 7},
    "self_attention_layer": None,
    "attention_layer": {"type": "EgoAttention", "feature_size": 64, "heads": 2},
    "output_layer": {"type": "MultiLayerPerceptron", "layers": [64, 64], "reshape": False},
}


class MultiLayerPerceptron(nn.Module):
    def __init__(self, inp: int, layers, out: int | None = None, reshape: bool = False):
        super().__init__()
        sizes = [inp] + list(layers)
        self.layers = nn.ModuleList([nn.Linear(sizes[i], sizes[i + 1]) for i in range(len(sizes) - 1)])
        self.predict = nn.Linear(sizes[-1], out) if out else None
        self.reshape = reshape

    def forward(self, x):
        if self.reshape:
            x = x.reshape(x.shape[0], -1)
        for layer in self.layers:
            x = F.relu(layer(x))
        return self.predict(x) if self.predict is not None else x


class EgoAttention(nn.Module):
    def __init__(self, feature_size: int = 64, heads: int = 2):
        super().__init__()
        self.f, self.h = feature_size, heads
        self.dph = feature_size // heads
        self.value_all = nn.Linear(feature_size, feature_size, bias=False)
        self.key_all = nn.Linear(feature_size, feature_size, bias=False)
        self.query_ego = nn.Linear(feature_size, feature_size, bias=False)
        self.attention_combine = nn.Linear(feature_size, feature_size, bias=False)

    def forward(self, ego, others, mask=None):
        b, n = others.shape[0], others.shape[1] + 1
        x = torch.cat((ego.view(b, 1, self.f), others), dim=1)
        k = self.key_all(x).view(b, n, self.h, self.dph).permute(0, 2, 1, 3)
        v = self.value_all(x).view(b, n, self.h, self.dph).permute(0, 2, 1, 3)
        q = self.query_ego(ego).view(b, 1, self.h, self.dph).permute(0, 2, 1, 3)
        # one query per env: the [1 x d] @ [d x n] products as broadcast multiply + reduce
        # (a batched GEMM of 16k 1x32x15 problems is ~20x slower on hipBLASLt)
        scores = (q * k).sum(-1, keepdim=True).transpose(-2, -1) / math.sqrt(self.dph)
        if mask is not None:
            scores = scores.masked_fill(mask.view(b, 1, 1, n).repeat(1, self.h, 1, 1), -1e9)
        p = F.softmax(scores, dim=-1)
        out = (p.transpose(-2, -1) * v).sum(-2, keepdim=True)
        return (self.attention_combine(out.reshape(b, self.f)) + ego.squeeze(1)) / 2, p


class EgoAttentionNetwork(nn.Module):
    def __init__(self, n_actions: int = 5, config: dict | None = None):
        super().__init__()
        c = config or EGO_ATTENTION_2H
        e, o, a, h = c["embedding_layer"], c["others_embedding_layer"], c["attention_layer"], c["output_layer"]
        self.presence_idx = c.get("presence_feature_idx", 0)
        self.ego_embedding = MultiLayerPerceptron(e["in"], e["layers"])
        self.others_embedding = MultiLayerPerceptron(o["in"], o["layers"])
        self.attention_layer = EgoAttention(a["feature_size"], a["heads"])
        self.output_layer = MultiLayerPerceptron(a["feature_size"], h["layers"], out=n_actions)

    def reset(self, generator: torch.Generator | None = None):
        """BaseModule._init_weights (models.py:24-33): Xavier-uniform weights, zero biases."""
        for m in self.modules():
            if isinstance(m, nn.Linear):
                bound = math.sqrt(6.0 / (m.in_features + m.out_features))
                with torch.no_grad():
                    m.weight.uniform_(-bound, bound, generator=generator)
                    if m.bias is not None:
                        m.bias.zero_()
        return self

    def packed_weights(self) -> torch.Tensor:
        """The weights in the ttrl_ego_attention_q packed layout (include/ttrl_mi355x.h), cached
        until a parameter changes (optimizer steps bump the tensors' versions)."""
        ps = [self.ego_embedding.layers[0], self.ego_embedding.layers[1], self.others_embedding.layers[0],
              self.others_embedding.layers[1]]
        a = self.attention_layer
        h = self.output_layer
        tensors = []
        for lin in ps[:2]:
            tensors += [lin.weight, lin.bias]
        for lin in ps[2:]:
            tensors += [lin.weight, lin.bias]
        tensors += [a.value_all.weight, a.key_all.weight, a.query_ego.weight, a.attention_combine.weight]
        tensors += [h.layers[0].weight, h.layers[0].bias, h.layers[1].weight, h.layers[1].bias,
                    h.predict.weight, h.predict.bias]
        key = tuple((t.data_ptr(), t._version) for t in tensors)
        if getattr(self, "_packed_key", None) != key:
            # matrices as [in][out] (Linear.weight transposed): coalesced reads in the kernels
            self._packed = torch.cat([(t.detach().t() if t.dim() == 2 else t.detach()).reshape(-1).float()
                                      for t in tensors]).contiguous()
            self._packed_key = key
        return self._packed

    def fused_supported(self) -> bool:
        e = self.ego_embedding
        return (len(e.layers) == 2 and e.layers[0].out_features == 64 and e.layers[1].out_features == 64
                and len(self.others_embedding.layers) == 2 and self.attention_layer.f == 64
                and len(self.output_layer.layers) == 2 and self.output_layer.layers[0].out_features == 64
                and self.output_layer.layers[1].out_features == 64 and self.output_layer.predict is not None
                and self.presence_idx == 0 and e.layers[0].in_features in (5, 7, 8))

    @torch.no_grad()
    def fused_q(self, x: torch.Tensor) -> torch.Tensor:
        """Q-values through the fused HIP forward (torch.ops.ttrl.ego_attention_q): inference only."""
        from . import ops
        return ops.T.ego_attention_q(x.float(), self.packed_weights(), self.attention_layer.h,
                                     self.output_layer.predict.out_features)

    def forward(self, x):
        # contiguous copies: hipBLASLt takes a 6x slower path on the strided [:, 1:, :] view
        ego, others = x[:, 0:1, :].contiguous(), x[:, 1:, :].contiguous()
        mask = x[:, :, self.presence_idx:self.presence_idx + 1] < 0.5
        att, _ = self.attention_layer(self.ego_embedding(ego), self.others_embedding(others), mask)
        return self.output_layer(att)


class EgoAttentionPolicy:
    """Batched DQN acting: Q = value_net(obs[E, V, F]); epsilon-greedy on the device."""

    def __init__(self, device, n_actions: int = 5, seed: int = 0, tau: float = 15000.0, temperature: float = 1.0,
                 final_temperature: float = 0.05, fused: bool = True, env_id_offset: int = 0):
        self.device = torch.device(device)
        # the global env id of obs row 0 (a data-parallel rank's shard offset, sharding.shard): the
        # fused draws are keyed on the global env, so every shard of one seed explores independently
        # and any split of the global batch draws the same action for the same env
        self.env_id_offset = int(env_id_offset)
        self.fused = fused  # acting through the fused HIP forward on a GPU (training uses the torch graph)
        g = torch.Generator(device="cpu")
        g.manual_seed(seed)
        self.value_net = EgoAttentionNetwork(n_actions).reset(g).to(self.device).eval()
        self.n_actions = n_actions
        self.tau, self.t0, self.t1 = tau, temperature, final_temperature
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed + 1)
        self.seed = int(seed) + 1  # the fused acting's Philox key
        self.time = 0  # EpsilonGreedy.time: the number of act() calls so far
        self.last_epsilon = None  # the epsilon of the latest act() (EpsilonGreedy.epsilon)

    def epsilon(self, t: int) -> float:
        """EpsilonGreedy.update (epsilon_greedy.py:37-48): epsilon at exploration time t."""
        return self.t1 + (self.t0 - self.t1) * math.exp(-t / self.tau)

    def fused_acting(self, obs: torch.Tensor) -> bool:
        return self.fused and obs.device.type == "cuda" and self.value_net.fused_supported()

    @torch.no_grad()
    def q_values(self, obs: torch.Tensor) -> torch.Tensor:
        if self.fused_acting(obs):
            return self.value_net.fused_q(obs)
        return self.value_net(obs)

    @torch.no_grad()
    def act(self, obs: torch.Tensor, t: int | None = None, epsilon: torch.Tensor | None = None,
            step: torch.Tensor | None = None, dtype: torch.dtype = torch.int64) -> torch.Tensor:
        """AbstractDQNAgent.act (dqn/abstract.py:65-83) for a batch: the exploration time is stepped
        first (step_time, :77-78), then EpsilonGreedy.update sets epsilon from it and the greedy
        action (np.argmax, first maximum), then the action is drawn from {a: epsilon / A +
        (1 - epsilon) [a == greedy]} (epsilon_greedy.py:32-48).  ``t``: the exploration time before
        this call (default: the policy's own counter).  ``epsilon`` / ``step`` (device scalars, float32 /
        int64) override the schedule and the draw counter: a captured graph refreshes them before
        every replay.  ``dtype``: the actions' index type (int64, or int32 -- the env's own, which
        env.step takes without a cast launch).

        On a GPU the forward, argmax and draw are ONE launch (ttrl::ego_attention_act, Philox
        keyed on (seed, env_id_offset + row, step)); elsewhere the torch forward with torch's generator."""
        t = self.time if t is None else int(t)
        self.time = t + 1
        self.last_epsilon = self.epsilon(self.time) if epsilon is None else epsilon
        if self.fused_acting(obs):
            from . import ops
            net = self.value_net
            act, _ = ops.T.ego_attention_act(obs.float(), net.packed_weights(), net.attention_layer.h,
                                             net.output_layer.predict.out_features,
                                             self.last_epsilon if epsilon is None else 0.0, self.seed, self.time,
                                             epsilon, step, int32_actions=dtype == torch.int32,
                                             env_offset=self.env_id_offset)
            return act if act.dtype == dtype else act.to(dtype)
        epsilon = self.last_epsilon
        q = self.value_net(obs)
        greedy = q.argmax(dim=1)
        e = obs.shape[0]
        u = torch.rand(e, device=self.device, generator=self.gen)
        rnd = torch.randint(0, self.n_actions, (e,), device=self.device, generator=self.gen)
        return torch.where(u < epsilon, rnd, greedy).to(dtype)
