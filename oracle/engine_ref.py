"""CPU replay of one actor-learner iteration (TEST INFRASTRUCTURE ONLY; also bench.py's
cpu_baseline leg).

Restates, on the synthetic env, the batched form of the reference worker loop:
  agent.py:52-67 (train: predict -> act -> observe -> new_random_game on terminal)
  agent.py:141-151 predict (q) / network.py:65-72 + assets/a3c.png (a3c) action draw
  agent.py:153-167 observe (reward clip, history add, update cadence, target sync)
  agent.py:169-207 batch_update (TD target) / assets/a3c.png n-step returns (a3c)
  agent.py:306-321 loss, per-tensor clip_by_norm(40), RMSProp apply (main.py:63-65)
with E envs in lock-step, the history kept as a ring of frames (history.py:13-24 order).
"""
import numpy as np

from . import philox as px
from . import ref_cpu as R
from .synthetic_env import SyntheticAtari, pool_frame, pool_frame84

EP_END_CHOICES = np.array([0.1, 0.01, 0.5], np.float32)   # main.py:68


class EngineRef:
    def __init__(self, params, num_envs, n_step, action_size, algo='a3c', start_lives=0, num_frames=64,
                 seed=123, env_id_base=0, world_size=1, random_start=30, action_repeat=1,
                 gamma=0.99, beta=0.01, learning_rate=0.0007, max_step=80_000_000, decay=0.99,
                 momentum=0.0, epsilon=0.1, clip_norm=40.0, literal_adv=False, ep_start=1.0,
                 ep_end_t=4_000_000, learn_start=32, target_q_update_step=40_000, discount=0.99,
                 dtype=np.float64, lstm=False, frame84=False, double_q=False, dqn_type='nips'):
        self.algo, self.A, self.E, self.n = algo, int(action_size), int(num_envs), int(n_step)
        self.seed = int(seed)
        self.k0, self.k1 = px.seed_key(seed)
        self.env = SyntheticAtari(seed, num_envs, num_frames, action_size, start_lives, random_start,
                                  action_repeat, env_id_base)
        self.ids = self.env.ids
        self.world = int(world_size)
        self.R = self.n + 4 + (1 if algo == 'q' else 0)
        self.ring = np.zeros((self.E, self.R, 84, 84), np.uint8)
        self.tau, self.global_step = 3, 0
        # the workers' base step: the loop counter of agent.py:55 starts at the global step read
        # in before_train (agent.py:34); worker step of rollout step t = wstep0 + tau - 3 + t
        self.wstep0 = 0
        self.params = {k: np.array(v, np.float32) for k, v in params.items()}
        self.tparams = {k: v.copy() for k, v in self.params.items()}
        self.ms = {k: np.ones_like(v) for k, v in self.params.items()}      # TF1 rms slot = 1
        self.mom = {k: np.zeros_like(v) for k, v in self.params.items()}
        self.h = dict(gamma=gamma, beta=beta, learning_rate=learning_rate, max_step=max_step, decay=decay,
                      momentum=momentum, epsilon=epsilon, clip_norm=clip_norm, literal_adv=literal_adv,
                      ep_start=ep_start, ep_end_t=ep_end_t, learn_start=learn_start,
                      target_q_update_step=target_q_update_step, discount=discount)
        self.dtype = dtype
        self.double_q = bool(double_q)     # agent.py:176-184 (q only)
        self.dqn_type = str(dqn_type).lower()   # network.py:30-54 trunk: 'nips' or 'nature' (a3c heads)
        if self.dqn_type == 'nature' and (algo != 'a3c' or lstm):
            raise ValueError('the nature trunk is an A3C Network trunk (network.py:30-42)')
        if self.double_q and algo != 'q':
            raise ValueError('double_q is a Q-learning option')
        # C5 LSTM head (ref_cpu.lstm_*): recurrent state carried across iterations, zeroed after a
        # terminal transition
        self.lstm = bool(lstm)
        if self.lstm and algo != 'a3c':
            raise ValueError('the LSTM head is an a3c head')
        U = R.LSTM_UNITS
        self.hc = (np.zeros((self.E, U), dtype), np.zeros((self.E, U), dtype))
        x0 = px.philox4x32(self.ids, 0, 0, 11, self.k0, self.k1)[0]
        self.ep_end = EP_END_CHOICES[x0 % 3]
        self._screens = {}
        # measurement mode M2 (a3c_engine_config.frame84): pool frames are pre-sized 84x84 screens
        self.frame84 = bool(frame84)
        self.cache_screens = True      # the fixed pool makes screens cacheable; bench turns it off

    # ---- screens of pool frames (cached: the pool is a fixed set) --------------------
    def _screen(self, f):
        return pool_frame84(self.seed, f) if self.frame84 else R.screen(pool_frame(self.seed, f))

    def screen_of(self, f):
        f = int(f)
        if not self.cache_screens:
            return self._screen(f)
        if f not in self._screens:
            self._screens[f] = self._screen(f)
        return self._screens[f]

    def reset(self):
        self.env.new_random_game()
        for e in range(self.E):
            s = self.screen_of(self.env.frame[e])
            for c in range(4):
                self.ring[e, c % self.R] = s
        self.tau, self.global_step, self.wstep0 = 3, 0, 0
        if self.lstm:
            self.hc = (np.zeros_like(self.hc[0]), np.zeros_like(self.hc[1]))

    def _step_z(self, st, carry):
        """per-step forward: z [E, zs] (and the LSTM head's new state when lstm)."""
        if not self.lstm:
            return R.forward(self.params, st, self.algo, self.dqn_type, dtype=self.dtype, keep=False)['z'], None
        P, dt = self.params, self.dtype
        h3 = R.forward(P, st, 'a3c', dtype=dt, keep=False)['h3']
        h, c, _ = R.lstm_cell(h3, carry[0], carry[1], P['lstm_w'], P['lstm_b'])
        z = np.concatenate([h @ P['p_w'].astype(dt) + P['p_b'].astype(dt),
                            h @ P['q_w'].astype(dt) + P['q_b'].astype(dt)], axis=1)
        return z, (h, c)

    def states(self, tau):
        """[E,84,84,4] NHWC u8 state s_tau (frames tau-3..tau)."""
        slots = [(tau - 3 + c) % self.R for c in range(4)]
        return np.ascontiguousarray(np.transpose(self.ring[:, slots], (0, 2, 3, 1)))

    def draw_words(self, t):
        """(u, rnd) of rollout step t: the Philox uniform the draw compares against and the
        random action of the epsilon branch (the words the engine's head kernel uses)."""
        tau = self.tau + t
        x = px.philox4x32(np.uint32(tau & 0xFFFFFFFF), np.uint32(tau >> 32), self.ids, px.P_ACTION,
                          self.k0, self.k1)
        return px.u01(x[0]), (x[1] % np.uint32(self.A)).astype(np.int32)

    def _draw(self, z, t):
        u, rnd = self.draw_words(t)
        if self.algo == 'a3c':
            pi, _, _ = R.softmax_stats(z[:, :self.A])
            return R.sample_categorical(pi.astype(np.float32), u), pi
        eps = self.eps(t)
        q = z[:, :self.A].astype(np.float32)
        greedy = np.argmax(q, axis=1).astype(np.int32)
        return np.where(u < eps, rnd, greedy).astype(np.int32), None

    def worker_step(self, t=0, tau=None):
        """agent.py:55's loop counter at rollout step t of the rollout starting at tau."""
        return self.wstep0 + (self.tau if tau is None else tau) - 3 + t

    def eps(self, t=0):
        """agent.py:142-144 at the worker step of rollout step t."""
        h = self.h
        step = float(self.worker_step(t))
        d = float(h['ep_end_t']) - max(0.0, step - float(h['learn_start']))
        ee = self.ep_end.astype(np.float64)
        return (ee + np.maximum(0.0, (float(h['ep_start']) - ee) * d / float(h['ep_end_t']))).astype(np.float32)

    def iterate(self, forced_actions=None, grads=True):
        """One iteration; returns a dict of everything the GPU engine exposes.  grads=False stops
        after the rollout and its targets (no batch forward / backward: for callers that
        back-propagate the engine's own saved activations instead); grads='losses' adds the
        independent batch forward and its losses, without the backward."""
        E, n, A, h = self.E, self.n, self.A, self.h
        acts = np.zeros((n, E), np.int32)
        sampled = np.zeros((n, E), np.int32)
        rewards = np.zeros((n, E), np.float32)
        rewards_raw = np.zeros((n, E), np.float32)
        terms = np.zeros((n, E), np.uint8)
        us = np.zeros((n, E), np.float32)
        epss = np.zeros((n, E), np.float32)
        zs, pis, frames = [], [], []
        h0c0 = self.hc
        for t in range(n):
            st = self.states(self.tau + t)
            z, hc = self._step_z(st, self.hc)
            a, pi = self._draw(z, t)
            us[t] = self.draw_words(t)[0]
            if self.algo == 'q':
                epss[t] = self.eps(t)
            sampled[t] = a
            acts[t] = a if forced_actions is None else forced_actions[t]
            zs.append(z)
            pis.append(pi)
            frame, reward, term = self.env.act(acts[t], is_training=True)
            rewards_raw[t] = reward
            rewards[t] = np.clip(reward, -1.0, 1.0)                      # agent.py:154
            terms[t] = term
            if self.lstm:
                keep = (1.0 - term.astype(np.float64))[:, None].astype(self.dtype)
                self.hc = (hc[0] * keep, hc[1] * keep)
            frames.append(frame.copy())
            for e in range(E):
                self.ring[e, (self.tau + t + 1) % self.R] = self.screen_of(frame[e])
            if term.any():
                self.env.new_random_game(term.astype(bool))
        states = np.concatenate([self.states(self.tau + t) for t in range(n)])      # b = t*E + e
        B = n * E
        out = dict(actions=acts, sampled=sampled, rewards=rewards, rewards_raw=rewards_raw, terminals=terms,
                   z=np.stack(zs), u=us, eps=epss, h0c0=h0c0,
                   pi=pis, frames=np.stack(frames), tau=self.tau)
        if self.algo == 'a3c':
            zb, _ = self._step_z(self.states(self.tau + n), self.hc)
            Rt = R.nstep_returns(rewards, terms, zb[:, A].astype(np.float32), h['gamma'])
            target = Rt.astype(np.float32)
            out['bootstrap_z'] = zb
        else:
            nxt = np.concatenate([self.states(self.tau + t + 1) for t in range(n)])
            qn = R.forward(self.tparams, nxt, 'q', dtype=self.dtype, keep=False)['z']
            if self.double_q:      # the online net's argmax on s_{t+1}, the target net's value there
                qo = R.forward(self.params, nxt, 'q', dtype=self.dtype, keep=False)['z']
                target = R.td_target_double(rewards.reshape(-1), terms.reshape(-1), qn.astype(np.float32),
                                            qo[:, :A].astype(np.float32), h['discount']).astype(np.float32)
                out['q_next_online'] = qo
            else:
                target = R.td_target(rewards.reshape(-1), terms.reshape(-1), qn.astype(np.float32),
                                     h['discount']).astype(np.float32)
        out['target'] = target.reshape(n, E)
        if not grads:
            return out
        if self.lstm:
            fwd = R.lstm_a3c_forward(self.params, states, n, h0c0[0], h0c0[1], terms, dtype=self.dtype)
            out['lstm'] = fwd['lstm']
        else:
            fwd = R.forward(self.params, states, self.algo, self.dqn_type, dtype=self.dtype)
        flat_acts = acts.reshape(-1)
        if self.algo == 'a3c':
            losses, dz = R.a3c_loss_and_dz(fwd['z'], flat_acts, target.reshape(-1).astype(self.dtype),
                                           h['beta'], h['literal_adv'])
        else:
            loss, dz = R.q_loss_and_dz(fwd['z'], flat_acts, target.reshape(-1).astype(self.dtype))
            losses = dict(loss=loss, q_mean=fwd['z'][np.arange(B), flat_acts].mean())
        if grads == 'losses':        # the independent forward's losses, no backward
            out.update(losses=losses, z_batch=fwd['z'])
            return out
        if self.lstm:
            g = R.lstm_a3c_backward(self.params, fwd, dz, terms)
        else:
            g = R.backward(self.params, fwd, dz, self.algo, self.dqn_type)
        grads = {k: np.asarray(v, np.float32).reshape(self.params[k].shape) for k, v in g.items()}
        sumsq = {k: np.float32(np.sum(v.astype(np.float64) ** 2)) for k, v in grads.items()}
        clipped = {k: R.clip_by_norm(v, h['clip_norm']) for k, v in grads.items()}
        out.update(losses=losses, grads=grads, sumsq=sumsq, clipped=clipped, z_batch=fwd['z'])
        return out

    def apply(self, clipped, advance_tau=True, tau=None):
        """RMSProp apply (+ q target sync).  advance_tau=False: the caller advances tau at
        rollout time (the engine's overlap pipeline, where rollout k+1 precedes apply k); tau: the
        applied rollout's start (default: the current tau, the synchronous order)."""
        return self.apply_sequence([clipped], advance_tau, tau)

    def apply_sequence(self, clipped_seq, advance_tau=True, tau=None):
        """The reference PS's rule for several workers (main.py:63-65, agent.py:321): every
        worker's clipped gradient is an RMSProp step of its own, applied in the given (arrival)
        order with this iteration's learning rate; then the target sync / counters once."""
        h = self.h
        lr = self.next_lr(tau)
        for clipped in clipped_seq:
            for k in self.params:
                R.rmsprop_apply(self.params[k], self.ms[k], self.mom[k], clipped[k].astype(np.float32), lr,
                                h['decay'], h['momentum'], h['epsilon'])
        self.finish_update(advance_tau)
        return lr

    def next_lr(self, tau=None):
        """Learning rate of the update of the rollout starting at tau: agent.py:393-395 evaluated
        at the worker's own step (agent.py:55 `self.step`, not the global T) of the rollout's last
        env step, whose observe runs the update (agent.py:162-163)."""
        h = self.h
        return R.learning_rate(self.worker_step(self.n - 1, tau), h['max_step'], h['learning_rate'])

    def finish_update(self, advance_tau=True):
        """Target sync (q, agent.py:166-167) and counter advance of an applied update."""
        h = self.h
        inc = self.n * self.E * self.world
        if self.algo == 'q':
            P = h['target_q_update_step']
            if (self.global_step + inc + 1) // P != (self.global_step + 1) // P:   # agent.py:166-167
                self.tparams = {k: v.copy() for k, v in self.params.items()}
        if advance_tau:
            self.tau += self.n
        self.global_step += inc
