//! rpkt-named header views over the records of `librpkt_gpu.so` (the MI355X batch
//! engine of this repository, C ABI `include/rpkt_gpu.h`).
//!
//! rpkt parses one frame at a time with generic views over `T: Buf`
//! (`rpkt/src/{ether,vlan,ipv4,udp,tcp}/generated.rs`): `X::parse(buf) -> Result<X<T>, T>`,
//! getters on `&self`, `payload(self) -> T`.  The engine walks that chain for a whole
//! device-resident batch and leaves one `rpkt_rec_t` per frame; the views here re-expose
//! a record under the same names, argument meaning and Ok/Err behaviour, so a receive
//! loop written against rpkt's chain reads the same after the batch call:
//!
//! ```ignore
//! let eth = EtherFrame::parse(Cursor::new(&rec)).unwrap();
//! let ip = Ipv4::parse(eth.payload()).unwrap();
//! let udp = Udp::parse(ip.payload()).unwrap();
//! assert!(ip.verify_checksum() && udp.verify_checksum());
//! ```
//!
//! `parse` returns `Ok` exactly when the reference `parse` at that position returned
//! `Ok` for the frame, and `Err(cursor)` (the cursor unchanged, as `ipv4/generated.rs:37,48`
//! return the buffer) otherwise.  The same mapping is implemented and tested in Python
//! (`rpkt_amd/views.py`, exercised by `tests/test_oracle_golden.py` and
//! `tests/test_oracle_ip6.py`).
pub mod ffi;

use core::net::Ipv4Addr;
pub use ffi::{rpkt_opts_t as Opts, rpkt_rec16_t as Rec16, rpkt_rec_t as Rec};

/// An API-level failure of a batch call (negative `rpkt_err` code).
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub struct Error(pub i32);

/// `Ok(())` for `RPKT_OK`, `Err(Error(code))` otherwise.
pub fn check(rc: i32) -> Result<(), Error> {
    if rc == ffi::RPKT_OK { Ok(()) } else { Err(Error(rc)) }
}

/// The name of a per-frame status (`rpkt_gpu_status_name`).
pub fn status_name(status: u8) -> &'static str {
    const NAMES: [&str; 21] = ["OK", "ETH_SHORT", "VLAN_SHORT", "NOT_IPV4", "IP_SHORT",
                               "IP_BAD_IHL", "IP_IHL_GT_LEN", "IP_TOT_LT_IHL", "IP_TOT_GT_LEN",
                               "L4_OTHER", "UDP_SHORT", "UDP_BAD_LEN", "TCP_SHORT",
                               "TCP_BAD_DOFF", "IP6_SHORT", "IP6_BAD_LEN", "IP6_EXT_SHORT",
                               "IP6_EXT_BAD_LEN", "IP6_FRAGMENT", "ICMP_EMPTY", "NO_INNER"];
    NAMES.get(status as usize).copied().unwrap_or("?")
}

/// rpkt/src/ether/mod.rs:12-36 (the values the path dispatches on).
pub mod ether_type {
    pub const IPV4: u16 = 0x0800;
    pub const ARP: u16 = 0x0806;
    pub const VLAN: u16 = 0x8100;
    pub const QINQ: u16 = 0x88a8;
    pub const IPV6: u16 = 0x86dd;
}

/// rpkt/src/ipv4/mod.rs:107-155 (the values the path dispatches on).
pub mod ip_protocol {
    pub const IPV6_HOP_BY_HOP_OPTS: u8 = 0;
    pub const ICMP: u8 = 1;
    pub const TCP: u8 = 6;
    pub const UDP: u8 = 17;
    pub const IPV6_ROUTE: u8 = 43;
    pub const IPV6_FRAG: u8 = 44;
    pub const AH: u8 = 51;
    pub const ICMPV6: u8 = 58;
    pub const IPV6_DEST_OPTS: u8 = 60;
}

#[derive(Clone, Copy, Debug, PartialEq, Eq)]
enum Stage { Ether, L3, L4, App }

/// The position the chain has reached in one frame (rpkt's `Cursor`, cursors.rs:34-60):
/// which header starts at `cursor()` and how many bytes `remaining()`.
#[derive(Clone, Copy, Debug)]
pub struct Cursor<'a> {
    rec: &'a Rec,
    stage: Stage,
    vlan_idx: u8,
    off: u32,
    len: u32,
}

impl<'a> Cursor<'a> {
    /// `Cursor::new(frame)`: the start of the chain of the frame this record describes.
    pub fn new(rec: &'a Rec) -> Self {
        Cursor { rec, stage: Stage::Ether, vlan_idx: 0, off: 0, len: rec.frame_len }
    }
    pub fn cursor(&self) -> usize { self.off as usize }
    pub fn remaining(&self) -> usize { self.len as usize }
    /// The cursor's bytes in `frame` (the frame the record was parsed from).
    pub fn chunk<'f>(&self, frame: &'f [u8]) -> &'f [u8] {
        &frame[self.cursor()..self.cursor() + self.remaining()]
    }
}

const fn ip_failed(s: u8) -> bool {
    matches!(s, ffi::RPKT_S_ETH_SHORT | ffi::RPKT_S_VLAN_SHORT | ffi::RPKT_S_NOT_IPV4
                | ffi::RPKT_S_IP_SHORT..=ffi::RPKT_S_IP_TOT_GT_LEN)
}

/// The record holds the IPv6 block (an RPKT_F_IPV6 parse dispatched it on 0x86DD).
pub fn is_ip6(r: &Rec) -> bool {
    let et = match r.n_vlan { 0 => r.ethertype, n => r.vlan_ethertype[(n - 1) as usize] };
    et == ether_type::IPV6
        && !matches!(r.status, ffi::RPKT_S_ETH_SHORT | ffi::RPKT_S_VLAN_SHORT | ffi::RPKT_S_NOT_IPV4)
}

/// EtherFrame (ether/generated.rs:17-67).
#[derive(Clone, Copy, Debug)]
pub struct EtherFrame<'a> { buf: Cursor<'a> }

impl<'a> EtherFrame<'a> {
    /// ether/generated.rs:34-41: Err iff chunk_len < 14.
    pub fn parse(buf: Cursor<'a>) -> Result<Self, Cursor<'a>> {
        if buf.stage != Stage::Ether || buf.rec.status == ffi::RPKT_S_ETH_SHORT {
            return Err(buf);
        }
        Ok(EtherFrame { buf })
    }
    pub fn dst_addr(&self) -> [u8; 6] { self.buf.rec.dst_addr }
    pub fn src_addr(&self) -> [u8; 6] { self.buf.rec.src_addr }
    pub fn ethertype(&self) -> u16 { self.buf.rec.ethertype }
    /// ether/generated.rs:63-67: advance(14).
    pub fn payload(self) -> Cursor<'a> {
        Cursor { stage: Stage::L3, vlan_idx: 0, off: 14, len: self.buf.len - 14, ..self.buf }
    }
}

/// VlanFrame (vlan/generated.rs:15-69), one per 802.1Q / 802.1ad tag the engine walked.
#[derive(Clone, Copy, Debug)]
pub struct VlanFrame<'a> { buf: Cursor<'a> }

impl<'a> VlanFrame<'a> {
    /// vlan/generated.rs:32-39: Ok for each tag the engine walked (at most RPKT_MAX_VLAN).
    pub fn parse(buf: Cursor<'a>) -> Result<Self, Cursor<'a>> {
        if buf.stage != Stage::L3 || buf.vlan_idx >= buf.rec.n_vlan { return Err(buf); }
        Ok(VlanFrame { buf })
    }
    fn tci(&self) -> u16 { self.buf.rec.vlan_tci[self.buf.vlan_idx as usize] }
    pub fn priority(&self) -> u8 { (self.tci() >> 13) as u8 }
    pub fn dei_flag(&self) -> bool { self.tci() & 0x1000 != 0 }
    pub fn vlan_id(&self) -> u16 { self.tci() & 0xfff }
    pub fn ethertype(&self) -> u16 { self.buf.rec.vlan_ethertype[self.buf.vlan_idx as usize] }
    /// vlan/generated.rs:63-69: advance(4).
    pub fn payload(self) -> Cursor<'a> {
        Cursor { vlan_idx: self.buf.vlan_idx + 1, off: self.buf.off + 4, len: self.buf.len - 4,
                 ..self.buf }
    }
}

/// Ipv4 (ipv4/generated.rs:17-127, 269-288).
#[derive(Clone, Copy, Debug)]
pub struct Ipv4<'a> { buf: Cursor<'a> }

impl<'a> Ipv4<'a> {
    /// ipv4/generated.rs:35-51 (its five checks, in order, decided by the engine).
    pub fn parse(buf: Cursor<'a>) -> Result<Self, Cursor<'a>> {
        let r = buf.rec;
        if buf.stage != Stage::L3 || buf.vlan_idx != r.n_vlan || ip_failed(r.status) || is_ip6(r) {
            return Err(buf);
        }
        Ok(Ipv4 { buf })
    }
    fn r(&self) -> &Rec { self.buf.rec }
    pub fn version(&self) -> u8 { self.r().ip_vhl >> 4 }
    pub fn dscp(&self) -> u8 { self.r().ip_tos >> 2 }
    pub fn ecn(&self) -> u8 { self.r().ip_tos & 3 }
    pub fn ident(&self) -> u16 { self.r().ip_ident }
    pub fn flag_reserved(&self) -> u8 { (self.r().ip_frag >> 15) as u8 }
    pub fn dont_frag(&self) -> bool { self.r().ip_frag & 0x4000 != 0 }
    pub fn more_frag(&self) -> bool { self.r().ip_frag & 0x2000 != 0 }
    pub fn frag_offset(&self) -> u16 { self.r().ip_frag & 0x1fff }
    pub fn ttl(&self) -> u8 { self.r().ip_ttl }
    pub fn protocol(&self) -> u8 { self.r().ip_protocol }
    pub fn checksum(&self) -> u16 { self.r().ip_checksum }
    pub fn header_len(&self) -> u8 { (self.r().ip_vhl & 0xf) * 4 }
    pub fn packet_len(&self) -> u16 { self.r().ip_packet_len }
    pub fn src_addr(&self) -> Ipv4Addr { Ipv4Addr::from(self.r().ip_src) }
    pub fn dst_addr(&self) -> Ipv4Addr { Ipv4Addr::from(self.r().ip_dst) }
    /// checksum::from_slice(header[0..header_len]) as the engine computed it.
    pub fn header_sum(&self) -> u16 { self.r().ip_sum }
    pub fn verify_checksum(&self) -> bool { self.header_sum() == 0xffff }
    /// ipv4/generated.rs:115-127: trim to packet_len, advance header_len.
    pub fn payload(self) -> Cursor<'a> {
        let len = self.packet_len() as u32 - self.header_len() as u32;
        Cursor { stage: Stage::L4, off: self.r().l4_off as u32, len, ..self.buf }
    }
}

/// Ipv6 (ipv6/generated.rs:22-216) over an IPv6 record: the record's IPv6 block
/// (include/rpkt_gpu.h, bytes 24..43); the addresses are read from the frame.
#[derive(Clone, Copy, Debug)]
pub struct Ipv6<'a> { buf: Cursor<'a> }

impl<'a> Ipv6<'a> {
    /// ipv6/generated.rs:40-51: Err iff chunk_len < 40 or payload_len + 40 > remaining.
    pub fn parse(buf: Cursor<'a>) -> Result<Self, Cursor<'a>> {
        let r = buf.rec;
        if buf.stage != Stage::L3 || buf.vlan_idx != r.n_vlan || !is_ip6(r)
            || matches!(r.status, ffi::RPKT_S_IP6_SHORT | ffi::RPKT_S_IP6_BAD_LEN) {
            return Err(buf);
        }
        Ok(Ipv6 { buf })
    }
    fn r(&self) -> &Rec { self.buf.rec }
    fn vtcfl(&self) -> u32 {
        self.r().ip_vhl as u32 | (self.r().ip_tos as u32) << 8 | (self.r().ip_packet_len as u32) << 16
    }
    pub fn version(&self) -> u8 { (self.vtcfl() >> 28) as u8 }
    pub fn traffic_class(&self) -> u8 { (self.vtcfl() >> 20) as u8 }
    pub fn flow_label(&self) -> u32 { self.vtcfl() & 0xfffff }
    pub fn payload_len(&self) -> u16 { self.r().ip_ident }
    pub fn next_header(&self) -> u8 { self.r().ip_frag as u8 }
    pub fn hop_limit(&self) -> u8 { (self.r().ip_frag >> 8) as u8 }
    /// Extension headers the engine walked before the upper-layer header.
    pub fn n_ext(&self) -> u8 { self.r().ip_ttl }
    /// The upper-layer protocol (the next_header where the extension walk stopped).
    pub fn upper_protocol(&self) -> u8 { self.r().ip_protocol }
    pub fn src_addr(&self, frame: &[u8]) -> core::net::Ipv6Addr {
        let o = self.r().l3_off as usize + 8;
        core::net::Ipv6Addr::from(<[u8; 16]>::try_from(&frame[o..o + 16]).unwrap())
    }
    pub fn dst_addr(&self, frame: &[u8]) -> core::net::Ipv6Addr {
        let o = self.r().l3_off as usize + 24;
        core::net::Ipv6Addr::from(<[u8; 16]>::try_from(&frame[o..o + 16]).unwrap())
    }
    /// The cursor past the extension headers (the upper-layer header, where Udp::parse /
    /// Tcp::parse apply): the end of the reference loop over DestOptions::parse,
    /// RoutingHeader::parse, ... and their payload().
    pub fn upper_layer(self) -> Cursor<'a> {
        let r = self.r();
        let end = r.l3_off as u32 + 40 + self.payload_len() as u32;
        Cursor { stage: Stage::L4, off: r.l4_off as u32, len: end - r.l4_off as u32, ..self.buf }
    }
}

fn l4_parse<'a>(buf: Cursor<'a>, proto: u8) -> Result<Cursor<'a>, Cursor<'a>> {
    let r = buf.rec;
    if buf.stage != Stage::L4 || r.status != ffi::RPKT_S_OK || r.ip_protocol != proto {
        return Err(buf);
    }
    Ok(buf)
}

/// Udp (udp/generated.rs:13-76).
#[derive(Clone, Copy, Debug)]
pub struct Udp<'a> { buf: Cursor<'a> }

impl<'a> Udp<'a> {
    /// udp/generated.rs:31-42.
    pub fn parse(buf: Cursor<'a>) -> Result<Self, Cursor<'a>> {
        l4_parse(buf, ip_protocol::UDP).map(|buf| Udp { buf })
    }
    pub fn src_port(&self) -> u16 { self.buf.rec.src_port }
    pub fn dst_port(&self) -> u16 { self.buf.rec.dst_port }
    pub fn checksum(&self) -> u16 { self.buf.rec.l4_checksum }
    pub fn packet_len(&self) -> u16 { self.buf.rec.l4_word6 }
    /// checksum::combine(&[pseudo_header, from_slice(udp)]) as the engine computed it.
    pub fn sum(&self) -> u16 { self.buf.rec.l4_sum }
    /// smoltcp's policy (the origin of checksum.rs): a zero checksum is "not computed",
    /// over IPv4 only (RFC 8200 section 8.1: mandatory over IPv6).
    pub fn verify_checksum(&self) -> bool {
        (self.checksum() == 0 && !is_ip6(self.buf.rec)) || self.sum() == 0xffff
    }
    /// udp/generated.rs:66-76: advance 8, trimmed to packet_len.
    pub fn payload(self) -> Cursor<'a> {
        let r = self.buf.rec;
        Cursor { stage: Stage::App, off: r.payload_off as u32, len: r.payload_len as u32,
                 ..self.buf }
    }
}

/// Tcp (tcp/generated.rs:16-131).
#[derive(Clone, Copy, Debug)]
pub struct Tcp<'a> { buf: Cursor<'a> }

impl<'a> Tcp<'a> {
    /// tcp/generated.rs:34-45.
    pub fn parse(buf: Cursor<'a>) -> Result<Self, Cursor<'a>> {
        l4_parse(buf, ip_protocol::TCP).map(|buf| Tcp { buf })
    }
    fn w6(&self) -> u16 { self.buf.rec.l4_word6 }
    pub fn src_port(&self) -> u16 { self.buf.rec.src_port }
    pub fn dst_port(&self) -> u16 { self.buf.rec.dst_port }
    pub fn seq_num(&self) -> u32 { self.buf.rec.tcp_seq }
    pub fn ack_num(&self) -> u32 { self.buf.rec.tcp_ack }
    pub fn reserved(&self) -> u8 { ((self.w6() >> 8) & 0xf) as u8 }
    pub fn cwr(&self) -> bool { self.w6() & 0x80 != 0 }
    pub fn ece(&self) -> bool { self.w6() & 0x40 != 0 }
    pub fn urg(&self) -> bool { self.w6() & 0x20 != 0 }
    pub fn ack(&self) -> bool { self.w6() & 0x10 != 0 }
    pub fn psh(&self) -> bool { self.w6() & 0x08 != 0 }
    pub fn rst(&self) -> bool { self.w6() & 0x04 != 0 }
    pub fn syn(&self) -> bool { self.w6() & 0x02 != 0 }
    pub fn fin(&self) -> bool { self.w6() & 0x01 != 0 }
    pub fn window_size(&self) -> u16 { self.buf.rec.tcp_window }
    pub fn checksum(&self) -> u16 { self.buf.rec.l4_checksum }
    pub fn urgent_pointer(&self) -> u16 { self.buf.rec.tcp_urgent }
    pub fn header_len(&self) -> u8 { ((self.w6() >> 12) * 4) as u8 }
    pub fn sum(&self) -> u16 { self.buf.rec.l4_sum }
    pub fn verify_checksum(&self) -> bool { self.sum() == 0xffff }
    /// tcp/generated.rs:125-131: advance header_len (no trim).
    pub fn payload(self) -> Cursor<'a> {
        let r = self.buf.rec;
        Cursor { stage: Stage::App, off: r.payload_off as u32, len: r.payload_len as u32,
                 ..self.buf }
    }
}

/// Views over a compact record (rpkt_gpu_parse_batch_compact): the cursors a lazy
/// receive loop reads its getters through, and the verdicts.
impl Rec16 {
    pub fn parsed_ok(&self) -> bool { self.status == ffi::RPKT_S_OK }
    /// Ipv4::parse returned Ok (the header is at l3_off, the payload at l4_off).
    pub fn ipv4_parsed(&self) -> bool { !ip_failed(self.status) && !self.is_ip6() }
    pub fn ip_sum_ok(&self) -> bool { self.verdict & 1 != 0 }
    /// The frame was dispatched to Ipv6::parse (verdict bit 2).
    pub fn is_ip6(&self) -> bool { self.verdict & 4 != 0 }
    /// status OK and the L4 sum verifies (a UDP checksum of 0 counts as verified).
    pub fn l4_sum_ok(&self) -> bool { self.verdict & 2 != 0 }
    /// (offset, length) of Udp::payload() / Tcp::payload() (status OK), else of
    /// Ipv4::payload().
    pub fn payload(&self) -> (usize, usize) { (self.payload_off as usize, self.payload_len as usize) }
}

/// The option walks of one frame (rpkt_gpu_options_batch / rpkt_gpu_parse_options_batch):
/// what TcpOptionsIter (tcp/generated.rs:1357-1484) and Ipv4OptionsIter
/// (ipv4/generated.rs:1595-1722) yield, with the getters of the last option of each kind.
impl Opts {
    fn tcp_has(&self, kind: u16) -> bool { self.tcp_kinds & (1 << kind) != 0 }
    fn ip_has(&self, kind: u16) -> bool { self.ip_kinds & (1 << kind) != 0 }
    /// Mss::mss
    pub fn mss(&self) -> Option<u16> { self.tcp_has(2).then_some(self.tcp_mss) }
    /// WindowScale::shift_count
    pub fn window_scale(&self) -> Option<u8> { self.tcp_has(3).then_some(self.tcp_wscale) }
    pub fn sack_permitted(&self) -> bool { self.tcp_has(4) }
    /// The first SACK block and the block count of the last Sack option.
    pub fn sack(&self) -> Option<(u32, u32, u8)> {
        self.tcp_has(5).then_some((self.tcp_sack_left, self.tcp_sack_right, self.tcp_sack_blocks))
    }
    /// Timestamp::{ts, ts_echo}
    pub fn timestamp(&self) -> Option<(u32, u32)> {
        self.tcp_has(6).then_some((self.tcp_ts, self.tcp_ts_echo))
    }
    /// RouteAlert::data
    pub fn route_alert(&self) -> Option<u16> { self.ip_has(4).then_some(self.ip_route_alert) }
    /// RecordRoute::{header_len, pointer}
    pub fn record_route(&self) -> Option<(u8, u8)> {
        self.ip_has(3).then_some((self.ip_rr_len, self.ip_rr_pointer))
    }
    /// CommercialSecurity::doi
    pub fn commercial_security_doi(&self) -> Option<u32> { self.ip_has(5).then_some(self.ip_cs_doi) }
    /// Strict/LooseSourceRoute::{pointer, dest_addr}
    pub fn source_route(&self) -> Option<(u8, Ipv4Addr)> {
        (self.ip_has(6) || self.ip_has(7)).then_some((self.ip_sr_pointer, Ipv4Addr::from(self.ip_sr_dest)))
    }
    /// Kind indices of the first min(count, 16) TCP options (4-bit codes, index + 1).
    pub fn tcp_kind_trace(&self) -> impl Iterator<Item = u8> + '_ {
        (0..self.tcp_count.min(16)).map(move |k| ((self.tcp_trace >> (4 * k)) & 15) as u8 - 1)
    }
    pub fn ip_kind_trace(&self) -> impl Iterator<Item = u8> + '_ {
        (0..self.ip_count.min(16)).map(move |k| ((self.ip_trace >> (4 * k)) & 15) as u8 - 1)
    }
}

/// A batch descriptor over device memory the caller owns (rpkt_batch_t).
pub fn strided_batch(frames_dev: *const u8, frames_bytes: u64, stride: u32, frame_len: u32,
                     n: u32) -> ffi::rpkt_batch_t {
    ffi::rpkt_batch_t { frames_dev, frames_bytes, offsets_dev: core::ptr::null(), stride,
                        frame_len, n, reserved: 0 }
}

/// Packed layout: frame i = [offsets[i], offsets[i + 1]) (n + 1 device u32 offsets).
pub fn packed_batch(frames_dev: *const u8, frames_bytes: u64, offsets_dev: *const u32,
                    n: u32) -> ffi::rpkt_batch_t {
    ffi::rpkt_batch_t { frames_dev, frames_bytes, offsets_dev, stride: 0, frame_len: 0, n,
                        reserved: 0 }
}

/// rpkt_gpu_parse_batch on `stream` (a hipStream_t, null = the null stream).
///
/// # Safety
/// `batch` must describe device memory valid for the call, and `recs_dev` must hold
/// `batch.n` records (16-byte aligned) on the same device.
pub unsafe fn parse_batch(batch: &ffi::rpkt_batch_t, flags: u32, recs_dev: *mut Rec,
                          stream: *mut core::ffi::c_void) -> Result<(), Error> {
    check(ffi::rpkt_gpu_parse_batch(batch, flags, recs_dev, core::ptr::null_mut(), 0, stream))
}

/// rpkt_gpu_parse_options_batch: records and option walks in one pass.
///
/// # Safety
/// As [`parse_batch`]; `opts_dev` must hold `batch.n` rpkt_opts_t (16-byte aligned).
pub unsafe fn parse_options_batch(batch: &ffi::rpkt_batch_t, flags: u32, recs_dev: *mut Rec,
                                  opts_dev: *mut Opts, stream: *mut core::ffi::c_void)
                                  -> Result<(), Error> {
    check(ffi::rpkt_gpu_parse_options_batch(batch, flags, recs_dev, opts_dev,
                                            core::ptr::null_mut(), 0, stream))
}
