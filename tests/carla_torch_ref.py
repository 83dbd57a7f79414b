"""Plain PyTorch fp32 (CPU) reference of one CaRL PPO minibatch (ac_ppo_carla.cpp:540-619 on the
carla_model.h agent): loss, full gradient, clip_grad_norm_ and one Adam step. Test infrastructure
only; tests/test_carla_oracle.py pins it to the LibTorch golden case carla_update."""
import numpy as np
import torch
import torch.nn.functional as F


def _tensors(L, p):
    """named_parameters() views of the flat vector (ppo_carla.h order), as leaf tensors"""
    t = {}
    names = ["action_space_high", "action_space_low"]
    for i in range(6):
        names += [f"cnn.{2 * i}.weight", f"cnn.{2 * i}.bias"]
    names += ["linear.0.weight", "linear.0.bias", "linear.2.weight", "linear.2.bias",
              "state_linear.0.weight", "state_linear.0.bias", "state_linear.2.weight", "state_linear.2.bias",
              "value_head.0.weight", "value_head.0.bias", "value_head.2.weight", "value_head.2.bias",
              "value_head.4.weight", "value_head.4.bias", "policy_head.0.weight", "policy_head.0.bias",
              "policy_head.2.weight", "policy_head.2.bias", "dist_mu.0.weight", "dist_mu.0.bias",
              "dist_sigma.0.weight", "dist_sigma.0.bias"]
    shapes = [(), ()]
    for i in range(6):
        shapes += [(L.conv_oc[i], L.conv_ic[i], L.conv_k[i], L.conv_k[i]), (L.conv_oc[i],)]
    shapes += [(512, 1280), (512,), (256, 512), (256,), (256, L.NM), (256,), (256, 256), (256,),
               (256, 256 + L.NV), (256,), (256, 256), (256,), (1, 256), (1,), (256, 256), (256,), (256, 256), (256,),
               (L.A, 256), (L.A,), (L.A, 256), (L.A,)]
    assert len(names) == L.ntensors
    for k, (name, shp) in enumerate(zip(names, shapes)):
        o, n = L.t_off[k], L.t_len[k]
        t[name] = torch.tensor(p[o:o + n].reshape(shp), dtype=torch.float32, requires_grad=bool(L.t_grad[k]))
    return names, t


def _beta_lp_ent(al, be, x):
    ab = al + be
    lp = torch.xlogy(al - 1.0, x) + torch.xlogy(be - 1.0, 1.0 - x) + torch.lgamma(ab) - torch.lgamma(al) - torch.lgamma(be)
    ent = (torch.lgamma(al) + torch.lgamma(be) - torch.lgamma(ab) - (2.0 - ab) * torch.digamma(ab)
           - ((al - 1.0) * torch.digamma(al) + (be - 1.0) * torch.digamma(be)))
    return lp.sum(1), ent.sum(1)


def update(L, p, bev, meas, vmeas, act, old_logp, adv, ret, old_v, clip=0.2, ent_coef=0.01, vf_coef=0.5,
           max_grad_norm=0.5, lr=3e-4, eps=1e-5, beta_min=1.0, norm_adv=True, clip_vloss=True, adv_stats=None,
           allreduce_grads=None):
    """adv_stats: (mean, std) to normalise with instead of this minibatch's own (the all-reduced
    statistics of ac_ppo_carla.cpp:561-580); allreduce_grads(list of grad tensors): called after
    backward and before clip_grad_norm_ (:608-616)."""
    names, t = _tensors(L, p)
    x = torch.tensor(bev).float() / 255.0
    for i in range(6):
        x = F.relu(F.conv2d(x, t[f"cnn.{2 * i}.weight"], t[f"cnn.{2 * i}.bias"], stride=L.conv_s[i]))
    x = torch.flatten(x, 1)
    s = F.relu(F.linear(torch.tensor(meas), t["state_linear.0.weight"], t["state_linear.0.bias"]))
    s = F.relu(F.linear(s, t["state_linear.2.weight"], t["state_linear.2.bias"]))
    h = F.relu(F.linear(torch.cat([x, s], 1), t["linear.0.weight"], t["linear.0.bias"]))
    feat = F.relu(F.linear(h, t["linear.2.weight"], t["linear.2.bias"]))
    v = F.relu(F.linear(torch.cat([feat, torch.tensor(vmeas)], 1), t["value_head.0.weight"], t["value_head.0.bias"]))
    v = F.relu(F.linear(v, t["value_head.2.weight"], t["value_head.2.bias"]))
    value = F.linear(v, t["value_head.4.weight"], t["value_head.4.bias"]).view(-1)
    pi = F.relu(F.linear(feat, t["policy_head.0.weight"], t["policy_head.0.bias"]))
    pi = F.relu(F.linear(pi, t["policy_head.2.weight"], t["policy_head.2.bias"]))
    al = F.softplus(F.linear(pi, t["dist_mu.0.weight"], t["dist_mu.0.bias"])) + beta_min
    be = F.softplus(F.linear(pi, t["dist_sigma.0.weight"], t["dist_sigma.0.bias"])) + beta_min
    hi, lo = t["action_space_high"], t["action_space_low"]
    a = (torch.tensor(act) - lo) / (hi - lo)
    a = torch.clamp(a, 1e-7, 1.0 + 1e-7)
    lp, ent = _beta_lp_ent(al, be, a)
    logratio = lp - torch.tensor(old_logp)
    ratio = logratio.exp()
    mb_adv = torch.tensor(adv)
    if norm_adv:
        if adv_stats is None:
            mb_adv = (mb_adv - mb_adv.mean()) / (mb_adv.std() + 1e-8)
        else:
            mb_adv = (mb_adv - adv_stats[0]) / (adv_stats[1] + 1e-8)
    pg = torch.max(-mb_adv * ratio, -mb_adv * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
    R, ov = torch.tensor(ret), torch.tensor(old_v)
    if clip_vloss:
        vc = ov + torch.clamp(value - ov, -clip, clip)
        vl = 0.5 * torch.max((value - R) ** 2, (vc - R) ** 2).mean()
    else:
        vl = 0.5 * ((value - R) ** 2).mean()
    loss = pg - ent_coef * ent.mean() + vf_coef * vl
    loss.backward()
    if allreduce_grads is not None:
        allreduce_grads([t[n].grad for n in names if t[n].grad is not None])
    with torch.no_grad():
        stats = [pg.item(), vl.item(), ent.mean().item(), (-logratio).mean().item(),
                 ((ratio - 1) - logratio).mean().item(), ((ratio - 1).abs() > clip).float().mean().item()]
    grad = np.zeros(L.P, np.float32)
    for k, n in enumerate(names):
        if t[n].grad is not None:
            grad[L.t_off[k]:L.t_off[k] + L.t_len[k]] = t[n].grad.numpy().reshape(-1)
    params = [t[n] for n in names]
    total = float(torch.nn.utils.clip_grad_norm_([q for q in params if q.requires_grad], max_grad_norm))
    opt = torch.optim.Adam([q for q in params if q.requires_grad], lr=lr, eps=eps)
    opt.step()
    new_p = np.concatenate([t[n].detach().numpy().reshape(-1) for n in names]).astype(np.float32)
    return grad, np.array(stats, np.float32), total, new_p, lp.detach().numpy(), value.detach().numpy()
