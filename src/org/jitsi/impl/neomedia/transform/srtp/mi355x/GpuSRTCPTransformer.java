/*
 * Drop-in for SRTCPTransformer (transform/srtp/SRTCPTransformer.java:30-208) on
 * the MI355X engine, with the reference's three constructors -- among them the
 * one DtlsPacketTransformer.initializeSRTCPTransformerFromRtp uses for
 * rtcp-mux (DtlsPacketTransformer.java:505-525).  NOT COMPILED IN THIS
 * REPOSITORY (no JDK); see INTEGRATION.md.
 */
package org.jitsi.impl.neomedia.transform.srtp.mi355x;

public class GpuSRTCPTransformer
    extends GpuTransformerBase
{
    /**
     * SRTCPTransformer(SRTPTransformer) (:50-54): shares the SRTP
     * transformer's factories (the contexts stay separate: one map per
     * transformer, SURVEY.md Q1).
     */
    public GpuSRTCPTransformer(GpuSRTPTransformer srtpTransformer)
    {
        this(srtpTransformer.forwardFactory, srtpTransformer.reverseFactory);
    }

    /** SRTCPTransformer(SRTPContextFactory) (:62-65) */
    public GpuSRTCPTransformer(GpuSRTPContextFactory factory)
    {
        this(factory, factory);
    }

    /** SRTCPTransformer(forwardFactory, reverseFactory) (:75-82) */
    public GpuSRTCPTransformer(GpuSRTPContextFactory forwardFactory, GpuSRTPContextFactory reverseFactory)
    {
        super(KIND_RTCP, forwardFactory, reverseFactory, null);
    }

    /** SRTCPTransformer.updateFactory (:92-117) */
    public void updateFactory(GpuSRTPContextFactory factory, boolean forward)
    {
        replaceFactory(factory, forward);
    }
}
