//! `Bote` / `Search` entry points over libbote_hip.so, keeping the reference
//! signatures (fantoch_bote/src/lib.rs:38-121, search.rs:262-319).  Sketch for
//! maintainers; not compiled here (no cargo in the image).
//! Written against the reference's real types: `Protocol` is neither `Copy`
//! nor `PartialEq` (fantoch_bote/src/protocol.rs:5-9), `ProtocolStats::insert`
//! takes (protocol, f, placement, stats) (protocol.rs:76-82), `Planet::regions`
//! returns an owned `Vec<Region>` (fantoch/src/planet/mod.rs:102), and the
//! crate is edition 2018 (no by-value array iteration).
use crate::hip;
use fantoch::metrics::Histogram;
use fantoch::planet::{Planet, Region};
use fantoch_bote::protocol::{ClientPlacement, Protocol, ProtocolStats};

/// A planet resident on one GPU.  Region ids are ranks of the region names,
/// so the device's (latency, id) order is the reference's (latency, Region)
/// order (fantoch/src/planet/mod.rs:122-140).
pub struct HipBote {
    dev: *mut hip::bote_planet,
    names: Vec<Region>, // sorted by name; index == id
}

impl HipBote {
    pub fn from(planet: &Planet, device: i32) -> Self {
        let mut names: Vec<Region> = planet.regions();
        names.sort();
        let r = names.len();
        let mut lat = vec![0u16; r * r];
        for (i, a) in names.iter().enumerate() {
            for (j, b) in names.iter().enumerate() {
                lat[i * r + j] = planet.ping_latency(a, b).expect("latency") as u16;
            }
        }
        let mut dev = std::ptr::null_mut();
        hip::check(unsafe { hip::bote_planet_create(lat.as_ptr(), r as u32, device, &mut dev) });
        HipBote { dev, names }
    }

    fn ids(&self, regions: &[Region]) -> Vec<u32> {
        regions
            .iter()
            .map(|x| self.names.binary_search(x).expect("region in planet") as u32)
            .collect()
    }

    /// Bote::leaderless (lib.rs:38-59)
    pub fn leaderless<'a>(&self, servers: &[Region], clients: &'a [Region], quorum_size: usize) -> Vec<(&'a Region, u64)> {
        let (s, c) = (self.ids(servers), self.ids(clients));
        let mut out = vec![0u64; c.len()];
        hip::check(unsafe {
            hip::bote_leaderless(self.dev, s.as_ptr(), s.len() as u32, c.as_ptr(), c.len() as u32,
                                 quorum_size as u32, out.as_mut_ptr())
        });
        clients.iter().zip(out).collect()
    }

    /// Bote::leader (lib.rs:67-89)
    pub fn leader<'a>(&self, leader: &Region, servers: &[Region], clients: &'a [Region], quorum_size: usize)
        -> Vec<(&'a Region, u64)> {
        let (s, c) = (self.ids(servers), self.ids(clients));
        let l = self.ids(std::slice::from_ref(leader))[0];
        let mut out = vec![0u64; c.len()];
        hip::check(unsafe {
            hip::bote_leader(self.dev, l, s.as_ptr(), s.len() as u32, c.as_ptr(), c.len() as u32,
                             quorum_size as u32, out.as_mut_ptr())
        });
        clients.iter().zip(out).collect()
    }

    /// Search::compute_stats (search.rs:262-319) for one configuration.
    pub fn compute_stats(&self, config: &[Region], all_clients: &[Region]) -> ProtocolStats {
        let (srv, cli) = (self.ids(config), self.ids(all_clients));
        let (n, nc) = (srv.len(), cli.len());
        let pos: Vec<u32> = (0..n as u32).collect();
        let stride = 5 * nc + 5 * n;
        let mut vals = vec![0u32; stride];
        let null64 = std::ptr::null_mut();
        hip::check(unsafe {
            hip::bote_eval(self.dev, srv.as_ptr(), n as u32, cli.as_ptr(), nc as u32, n as u32, pos.as_ptr(), 0,
                           1, std::ptr::null(), vals.as_mut_ptr(), std::ptr::null_mut(), null64, null64,
                           std::ptr::null_mut(), std::ptr::null_mut(), std::ptr::null_mut(),
                           std::ptr::null_mut())
        });
        // slot layout (include/bote_hip.h, bote_eval): af1 ff1 af2 ff2 e for
        // Input (nc values each), then the same five for Colocated (n values)
        let max_f = std::cmp::min(n / 2, 2);
        // slot k -> (protocol, f); Protocol is not Copy, so it is built per use
        fn slot_protocol(k: usize) -> Protocol {
            match k {
                0 | 2 => Protocol::Atlas,
                1 | 3 => Protocol::FPaxos,
                _ => Protocol::EPaxos,
            }
        }
        const SLOT_F: [usize; 5] = [1, 1, 2, 2, 0];
        let mut stats = ProtocolStats::new();
        let placements = [(ClientPlacement::Input, 0, nc), (ClientPlacement::Colocated, 5 * nc, n)];
        for &(placement, base, len) in placements.iter() {
            for k in 0..5 {
                let f = SLOT_F[k];
                if k != 4 && f > max_f {
                    continue;
                }
                let v = &vals[base + k * len..base + (k + 1) * len];
                let hist = Histogram::from(v.iter().map(|x| *x as u64));
                stats.insert(slot_protocol(k), f, placement, hist);
            }
        }
        stats
    }

    /// The multi-GPU exhaustive search (bote_search_create/launch/result):
    /// colex ranks of n-subsets of `servers` sharded over this planet and
    /// `others`, merged on this planet's device; records ascending by
    /// (key, rank).  All host work (shard bounds, chunk tables) happens in
    /// `HipSearch::new`; every `run` is device work only.  `keys` selects the
    /// key set (0: compute_stats' keys; 1: + Tempo tiny/write and FPaxos all
    /// leaders, BASELINE config 5).
    pub fn search<'b>(&'b self, others: &[&'b HipBote], servers: &[Region], clients: &[Region], n: usize,
                      objectives: &[hip::bote_objective], k: usize, rp: &hip::bote_ranking_params, keys: u32)
        -> HipSearch<'b> {
        let (s, c) = (self.ids(servers), self.ids(clients));
        let mut planets: Vec<*const hip::bote_planet> = vec![self.dev as *const _];
        planets.extend(others.iter().map(|b| b.dev as *const _));
        let total = unsafe { hip::bote_binomial(s.len() as u32, n as u32) };
        let mut h: *mut hip::bote_search = std::ptr::null_mut();
        hip::check(unsafe {
            hip::bote_search_create(planets.as_ptr(), planets.len() as u32, s.as_ptr(), s.len() as u32, c.as_ptr(),
                                    c.len() as u32, n as u32, 0, total, objectives.as_ptr(), objectives.len() as u32,
                                    k as u32, rp, 1, keys, &mut h)
        });
        HipSearch { h, n_obj: objectives.len(), k, _planets: std::marker::PhantomData }
    }

    /// One-shot form (bote_search_topk): create, run once, destroy.
    pub fn search_topk(&self, others: &[&HipBote], servers: &[Region], clients: &[Region], n: usize,
                       objectives: &[hip::bote_objective], k: usize, rp: &hip::bote_ranking_params)
        -> (Vec<Vec<hip::bote_topk_record>>, u64, u64) {
        self.search(others, servers, clients, n, objectives, k, rp, 0).run()
    }
}

/// A persistent multi-device search (bote_search_*); it borrows the planets.
pub struct HipSearch<'a> {
    h: *mut hip::bote_search,
    n_obj: usize,
    k: usize,
    _planets: std::marker::PhantomData<&'a HipBote>,
}

impl<'a> HipSearch<'a> {
    /// Launch every shard and the merge (device work only), then read the
    /// merged top-K lists, the valid count and the digest.
    pub fn run(&self) -> (Vec<Vec<hip::bote_topk_record>>, u64, u64) {
        let (no, k) = (self.n_obj, self.k);
        let mut recs = vec![hip::bote_topk_record { key: 0, rank: 0 }; no * k];
        let mut cnt = vec![0u32; no];
        let (mut valid, mut digest) = (0u64, 0u64);
        hip::check(unsafe { hip::bote_search_launch(self.h) });
        hip::check(unsafe {
            hip::bote_search_result(self.h, recs.as_mut_ptr(), cnt.as_mut_ptr(), &mut valid, &mut digest)
        });
        let tops = (0..no).map(|o| recs[o * k..o * k + cnt[o] as usize].to_vec()).collect();
        (tops, valid, digest)
    }
}

impl<'a> Drop for HipSearch<'a> {
    fn drop(&mut self) {
        unsafe {
            hip::bote_search_destroy(self.h);
        }
    }
}

impl Drop for HipBote {
    fn drop(&mut self) {
        unsafe {
            hip::bote_planet_destroy(self.dev);
        }
    }
}
