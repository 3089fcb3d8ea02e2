/*
 * What GpuSRTPTransformer and GpuSRTCPTransformer share: a SinglePacketTransformer
 * (transform/SinglePacketTransformer.java:33-217) whose per-packet
 * transform(RawPacket) / reverseTransform(RawPacket) run on the MI355X engine.
 * Not compiled in this repository (no JDK); see INTEGRATION.md.
 *
 * Per packet (what every reference caller does: the connectors' 1-element
 * arrays, RTPConnectorInputStream.java:425-452 / RTPConnectorOutputStream.java
 * :268-300, and DtlsPacketTransformer.transformSrtp, :1544-1564): one
 * srtp_rawpacket_transform_one through the process's aggregator, which puts the
 * packets of all concurrently calling threads into shared GPU bundles and
 * returns each caller its own packet.  Arrays of more than one packet go
 * through srtp_rawpacket_transform with SinglePacketTransformer's
 * abort-on-throw: up to 8192 packets none of which can throw share the
 * aggregator's bundles with every other thread's packets, other arrays run as
 * one bundle of their own; an array of one takes the inherited loop over the
 * per-packet call.  Threads that keep many packets in flight use
 * GpuPacketQueue instead.
 */
package org.jitsi.impl.neomedia.transform.srtp.mi355x;

import org.jitsi.impl.neomedia.*;
import org.jitsi.impl.neomedia.transform.*;
import org.jitsi.util.function.*;

abstract class GpuTransformerBase
    extends SinglePacketTransformer
{
    static final int KIND_RTP = 0, KIND_RTCP = 1;

    /* include/srtp_mi355x.h SRTP_STATUS_* */
    static final int STATUS_OK = 0, STATUS_ERR_MALFORMED = 6, STATUS_SKIPPED = 9;

    GpuSRTPContextFactory forwardFactory;
    GpuSRTPContextFactory reverseFactory;

    final int tid;

    final Predicate<RawPacket> packetPredicate;

    private long exceptionsInBatchTransform, exceptionsInBatchReverseTransform;

    GpuTransformerBase(int kind, GpuSRTPContextFactory forwardFactory,
                       GpuSRTPContextFactory reverseFactory, Predicate<RawPacket> packetPredicate)
    {
        super(packetPredicate);
        this.packetPredicate = packetPredicate;
        this.forwardFactory = forwardFactory;
        this.reverseFactory = reverseFactory;
        tid = SrtpMi355x.check(SrtpMi355x.transformerCreate(SrtpMi355x.dispatch(), kind,
                                                            forwardFactory.id, reverseFactory.id));
    }

    /**
     * SRTPTransformer.setContextFactory / SRTCPTransformer.updateFactory
     * (SRTPTransformer.java:100-125): the replaced factory is closed, the
     * contexts stay (SDES rekey).
     */
    void replaceFactory(GpuSRTPContextFactory factory, boolean forward)
    {
        synchronized (this)
        {
            SrtpMi355x.check(SrtpMi355x.transformerSetFactory(SrtpMi355x.dispatch(), tid, factory.id,
                                                              forward));
            if (forward)
                forwardFactory = factory;
            else
                reverseFactory = factory;
        }
    }

    /** SRTPTransformer.close() (:132-150): both factories and every context. */
    @Override
    public void close()
    {
        SrtpMi355x.transformerClose(SrtpMi355x.dispatch(), tid);
    }

    @Override
    public RawPacket transform(RawPacket pkt)
    {
        return one(pkt, false);
    }

    @Override
    public RawPacket reverseTransform(RawPacket pkt)
    {
        return one(pkt, true);
    }

    /**
     * SRTPTransformer.transform / reverseTransform (:185-219): null for a
     * dropped packet, an exception where SRTPCryptoContext throws (the packet
     * keeps what was done to it), else the packet, written back in place or
     * moved to a new buffer where RawPacket.append / grow reallocate.
     */
    private RawPacket one(RawPacket pkt, boolean reverse)
    {
        int st = SrtpMi355x.check(SrtpMi355x.transformOne(SrtpMi355x.aggregator(), reverse, tid, pkt));
        if (st == STATUS_ERR_MALFORMED)
            throw new IllegalArgumentException("SRTP: malformed packet");
        return st == STATUS_OK || st == STATUS_SKIPPED ? pkt : null;
    }

    @Override
    public RawPacket[] transform(RawPacket[] pkts)
    {
        return pkts != null && pkts.length > 1 ? batch(pkts, false) : super.transform(pkts);
    }

    @Override
    public RawPacket[] reverseTransform(RawPacket[] pkts)
    {
        return pkts != null && pkts.length > 1 ? batch(pkts, true) : super.reverseTransform(pkts);
    }

    /** SinglePacketTransformer.java:121-216 over the whole array in one bundle. */
    private RawPacket[] batch(RawPacket[] pkts, boolean reverse)
    {
        int[] skip = null;
        if (packetPredicate != null)
        {
            skip = new int[pkts.length];
            for (int i = 0; i < pkts.length; i++)
                if (pkts[i] != null && !packetPredicate.test(pkts[i]))
                    skip[i] = 1;
        }
        int r = SrtpMi355x.check(SrtpMi355x.transformPackets(SrtpMi355x.dispatch(), SrtpMi355x.aggregator(),
                                                             reverse, tid, pkts, skip));
        if (r > 0)
        {
            if (reverse)
                exceptionsInBatchReverseTransform++;
            else
                exceptionsInBatchTransform++;
            throw new IllegalArgumentException("Failed to " + (reverse ? "reverse-" : "")
                                               + "transform RawPacket(s)! (element " + (r - 1) + ")");
        }
        return pkts;
    }
}
